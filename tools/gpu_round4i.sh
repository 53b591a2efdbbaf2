#!/bin/bash
# Round-4 (i): bisect further (stream pool off): (1) the handle-churn test then the agent's compute_trajectory test;
# if that passes, (2) every in-flight test then compute_trajectory. A segfault ends the call.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
run() {  # name, pytest selection...
  local n=$1; shift
  timeout -k 10 400 env DDMI_STREAM_POOL=0 python -u -m pytest "$@" -v -m gpu -x --timeout 300 --timeout-method thread \
    > gpurun_out/order_$n.log 2>&1
  local rc=$?; echo "[order_$n] rc=$rc"; tail -2 gpurun_out/order_$n.log; return $rc
}
run churn_agent tests/test_inflight_gpu.py::test_handle_churn_then_two_stream_replay \
  tests/test_agent.py::test_compute_trajectory_matches_oracle || exit $?
run inflight_agent tests/test_inflight_gpu.py tests/test_agent.py::test_compute_trajectory_matches_oracle || exit $?
