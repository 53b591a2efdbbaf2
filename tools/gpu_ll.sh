#!/bin/bash
# launch-shape breakdowns for a list of env settings: gpu_ll.sh "ENV=1" "ENV=2" ...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 300 python tools/launch_log.py --gemm ${GEMM:-f16x3} --out gpurun_out/ll_$i.md > gpurun_out/ll_$i.log 2>&1
  rc=$?; echo "[$e] rc=$rc"; head -1 gpurun_out/ll_$i.md; grep "conv_gemm total" gpurun_out/ll_$i.md
  [ $rc -ne 0 ] && exit $rc
done
exit 0
