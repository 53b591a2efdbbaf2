#!/bin/bash
# round 5s: conv_x6 small-grid form (8 x 8 x 64, 4 waves) forced on the B = 64 trunk shapes vs the routed forms
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for shp in img.l1.3x3 img.l2.3x3 img.l3.3x3 img.l4.3x3 lid.l1.3x3 lid.l2.3x3 lid.l3.3x3 fx.l3.c128; do
  for cfg in "DDMI_X6_SMALL=1" "DDMI_X6_SMALL=2"; do
    out=$(env $cfg timeout -k 5 60 tools/micro/conv_bench ${REPS:-30} $shp 2>&1)
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc $shp [$cfg]"; echo "$out"; exit $rc; }
    echo "$out" | awk -v s="$shp" -v c="[$cfg]" '$1 == s { print c " " $0 }'
  done
done > gpurun_out/r5s_small.txt
rc=$?; cat gpurun_out/r5s_small.txt; exit $rc
