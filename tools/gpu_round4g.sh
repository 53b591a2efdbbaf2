#!/bin/bash
# Round-4 (g): localise the hipGraphLaunch segfault of the reproducing order (runner -> inflight -> agent tests, stream
# pool off) with runtime toggles: (1) the HIP runtime's graph packet capture off (DEBUG_CLR_GRAPH_PACKET_CAPTURE=0);
# if that passes, (2) single-stream graphs only (DDMI_STREAMS=0). A segfault ends the call (nothing runs after it).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
run() {  # name, env...
  local n=$1; shift
  timeout -k 10 400 env DDMI_STREAM_POOL=0 "$@" python -u -m pytest tests/test_runner.py tests/test_inflight_gpu.py \
    tests/test_agent.py -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/order_$n.log 2>&1
  local rc=$?; echo "[order_$n] rc=$rc"; tail -2 gpurun_out/order_$n.log; return $rc
}
run nopc DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 || exit $?
run single DDMI_STREAMS=0 || exit $?
