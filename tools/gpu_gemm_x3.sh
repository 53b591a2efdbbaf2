#!/bin/bash
# GPU box: GPT-shaped GEMM microbenchmark under rocprofv3 kernel trace, once per env setting given as arguments.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 180 rocprofv3 --kernel-trace -f csv -d "$R/gpurun_out/gx$i" -o run -- python3 "$R/tools/micro/gemm_x3_bench.py" > "$R/gpurun_out/gx$i.log" 2>&1
  rc=$?; echo "[$e] rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
