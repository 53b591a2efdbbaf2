#!/bin/bash
# Round-4 (b): the training-head GPU tests, then the handle-lifetime investigation with the dbg library
# (host SIGSEGV backtrace + handle / graph lifecycle trace) in the round-3 reproducing order with the stream pool
# off. A segfault in the last step is the expected finding; nothing runs after it.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -3 "gpurun_out/$name.log"
  return $rc
}
run train_tests 600 python -u -m pytest tests/test_train_loss.py -v -m gpu -x --timeout 300 --timeout-method thread || exit $?
run order_dbg 600 env DDMI_STREAM_POOL=0 DDMI_LIB=$R/diffusiondrive_amd/_variants/libddmi_dbg.so python -u -m pytest \
  tests/test_runner.py tests/test_inflight_gpu.py tests/test_agent.py -v -m gpu -x --timeout 300 --timeout-method thread
