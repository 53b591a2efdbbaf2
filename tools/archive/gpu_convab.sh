#!/bin/bash
# conv micro-benchmark A/B over environments (tools/micro/conv_bench; exact shape names):
#   SHAPES="img.l2.3x3 lid.l3.3x3" tools/archive/gpu_convab.sh "" "DDMI_X6_CFG=1" ...
# prints "[env] <shape> ms TF/s ..." per shape and environment
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for shp in ${SHAPES}; do
  for cfg in "$@"; do
    out=$(env $cfg timeout -k 5 60 tools/micro/conv_bench ${REPS:-30} $shp 2>&1)
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc $shp [$cfg]"; echo "$out"; exit $rc; }
    echo "$out" | awk -v s="$shp" -v c="[$cfg]" '$1 == s { print c " " $0 }'
  done
done
