#!/bin/bash
# conv microbenchmark: the product library against variant builds on one box (tools/micro/<variant>/conv_bench),
# shape filter $F (default 3x3). usage: gpu_variants.sh x6o2 x6o4 ...
set -u
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
for v in base "$@" base; do
  b=tools/micro/conv_bench; [ "$v" != base ] && b=tools/micro/$v/conv_bench
  timeout -k 10 100 $b 10 ${F:-3x3} > gpurun_out/var.log 2>&1 || { cat gpurun_out/var.log; exit 1; }
  echo "== $v"; grep -v "^shape" gpurun_out/var.log | awk '{printf "%s %s %s | ", $1, $2, $5} END {print ""}'
done
