#!/bin/bash
# GPU box: conv microbenchmark under each DDMI_X6_CFG value given. Stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for c in "$@"; do
  echo "== DDMI_X6_CFG=$c"
  DDMI_X6_CFG=$c timeout -k 10 120 tools/micro/conv_bench 10 ${SHAPE:-3x3} > gpurun_out/x6cfg_$c.log 2>&1
  rc=$?; grep -v "amdgpu.ids" gpurun_out/x6cfg_$c.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
