#!/bin/bash
# Round-4 (h): bisect the reproducing order (stream pool off) at the test level. (1) runner -> inflight -> the agent's
# compute_trajectory test alone (the agent's GPU feature-builder tests deselected); if that passes, (2) the extended
# pure-HIP reproducer (4 fork / join pairs per graph, memset nodes; pool off; streams kept / all re-created), then
# (3) inflight -> agent (all) without the runner tests. A segfault ends the call.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
run() {  # name, pytest selection...
  local n=$1; shift
  timeout -k 10 400 env DDMI_STREAM_POOL=0 python -u -m pytest "$@" -v -m gpu -x --timeout 300 --timeout-method thread \
    > gpurun_out/order_$n.log 2>&1
  local rc=$?; echo "[order_$n] rc=$rc"; tail -2 gpurun_out/order_$n.log; return $rc
}
run nofeat tests/test_runner.py tests/test_inflight_gpu.py tests/test_agent.py::test_compute_trajectory_matches_oracle || exit $?
for a in "0 4 1 0" "0 4 1 1"; do
  set -- $a
  timeout -k 10 200 tools/repro/graph_churn 100 $1 64 $4 $2 $3 > gpurun_out/churn_f$2m$3a$4.log 2>&1; rc=$?
  echo "[churn pool=$1 forks=$2 memset=$3 all=$4] rc=$rc"; tail -1 gpurun_out/churn_f$2m$3a$4.log; [ $rc -ne 0 ] && exit $rc
done
run norunner tests/test_inflight_gpu.py tests/test_agent.py || exit $?
