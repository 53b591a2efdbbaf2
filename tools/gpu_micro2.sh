#!/bin/bash
# GPU box: conv microbenchmark over env variants, compact (shape filter $F, default all).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for v in "$@"; do
  env $v timeout -k 10 120 tools/micro/conv_bench 10 ${F:-} > "gpurun_out/m2.log" 2>&1
  rc=$?; echo "== $v"; grep -v "^shape" gpurun_out/m2.log | awk '{printf "%s %s %s | ", $1, $2, $3} END {print ""}'
  if [ $rc -ne 0 ]; then cat gpurun_out/m2.log; echo "rc=$rc: stopping"; exit $rc; fi
done
