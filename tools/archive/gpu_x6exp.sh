#!/bin/bash
# conv_x6 epilogue experiments on the conv micro-benchmark: diagnostic knobs (DDMI_X6_DIAG: 1 = no residual read,
# 2 = no output store). (Round 3 also swept a first-round stagger, DDMI_X6_STAGGER, since removed: profiles/round3_d_x6_epilogue_exp.txt.)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
out=gpurun_out/x6exp.log; : > $out
for shp in ${SHAPES:-img.l1.3x3 img.l2.3x3 img.l3.3x3 img.l4.3x3 lid.l1.3x3}; do
  for cfg in "0 0" "0 1" "0 2" "0 3"; do
    set -- $cfg
    r=$(DDMI_X6_DIAG=$2 timeout -k 5 60 tools/micro/conv_bench ${REPS:-30} $shp 2>&1 | tail -1)
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc $shp $cfg"; exit $rc; }
    echo "diag=$2 $r" | tee -a $out
  done
done
