#!/bin/bash
# GPU box: conv microbenchmark (all shapes) against two library builds (tools/micro/ab_old, ab_new), alternating.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for v in old new old new; do
  LD_LIBRARY_PATH=tools/micro/ab_$v timeout -k 10 120 tools/micro/conv_bench 20 > gpurun_out/cab_$v.log 2>&1
  rc=$?; echo "== $v rc=$rc"; grep -v "amdgpu.ids" gpurun_out/cab_$v.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
