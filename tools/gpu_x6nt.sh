#!/bin/bash
# conv_x6 knobs on the conv micro-benchmark, per trunk shape: activation cache policy (DDMI_X6_NT 0-3) and the
# relaxed step barrier with a spare ring slot (DDMI_X6_RELAX=1), each read per dispatch.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
out=gpurun_out/x6nt.log; : > $out
for shp in ${SHAPES:-img.l1.3x3 img.l2.3x3 img.l3.3x3 img.l4.3x3 lid.l1.3x3 lid.l3.3x3 lid.l4.3x3}; do
  for v in "DDMI_X6_NT=0" "DDMI_X6_NT=1" "DDMI_X6_NT=3" "DDMI_X6_RELAX=1" "DDMI_X6_CFG=3" "DDMI_X6_CFG=3 DDMI_X6_NT=1" "DDMI_X6_NT=0"; do
    r=$(env $v timeout -k 5 60 tools/micro/conv_bench ${REPS:-20} $shp 2>&1 | tail -1)
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc $shp $v"; exit $rc; }
    echo "[$v] $r" | tee -a $out
  done
done
