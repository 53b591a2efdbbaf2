#!/bin/bash
# Round-4 (a): tools/gpu_all.sh (GPU tests, bench, rocprof trace), then the handle-lifetime investigation:
# the minimal HIP reproducer (tools/repro/graph_churn.hip) with the stream pool on and off, then the round-3
# reproducing test order (runner -> in-flight -> agent) with the library's pool off. Stops at the first abnormal
# exit (a segfault here is the finding).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
bash tools/gpu_all.sh || exit $?
bash tools/gpu_x6var.sh || exit $?
cd "$R"
run() {  # run <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -3 "gpurun_out/$name.log"
  return $rc
}
run churn_pool1 150 tools/repro/graph_churn 200 1 64 || exit $?
run churn_pool0 150 tools/repro/graph_churn 200 0 64 || exit $?
run order_pool0 600 env DDMI_STREAM_POOL=0 python -u -m pytest tests/test_runner.py tests/test_inflight_gpu.py tests/test_agent.py \
  -v -m gpu -x --timeout 300 --timeout-method thread || exit $?
