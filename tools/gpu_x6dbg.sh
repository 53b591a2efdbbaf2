#!/bin/bash
# GPU box: conv_x6 ablations (DDMI_X6_DBG bits) on the conv microbenchmark. Stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for d in ${DBGS:-0 1 2 4 8 16}; do
  echo "== DDMI_X6_DBG=$d"
  DDMI_X6_DBG=$d timeout -k 10 120 tools/micro/conv_bench 10 ${SHAPE:-3x3} > gpurun_out/x6dbg_$d.log 2>&1
  rc=$?; grep -v "amdgpu.ids" gpurun_out/x6dbg_$d.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
