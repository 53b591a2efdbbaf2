#!/bin/bash
# Round-4 (n): the reproducing order (stream pool off) with (1) the captured graphs kept alive beside their execs
# (DDMI_KEEP_GRAPH=1); if that passes, (2) single-stream graphs (DDMI_STREAMS=0). A segfault ends the call.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
run() {  # name, env...
  local n=$1; shift
  timeout -k 10 400 env DDMI_STREAM_POOL=0 "$@" python -u -m pytest tests/test_runner.py tests/test_inflight_gpu.py \
    tests/test_agent.py::test_compute_trajectory_matches_oracle -v -m gpu -x --timeout 300 --timeout-method thread \
    > gpurun_out/order_$n.log 2>&1
  local rc=$?; echo "[order_$n] rc=$rc"; tail -2 gpurun_out/order_$n.log; return $rc
}
# (4n, first step: the captured graphs kept alive beside their execs - DDMI_KEEP_GRAPH, since removed - still faulted)
run single DDMI_STREAMS=0 || exit $?
