#!/bin/bash
# Validation of a default change: the reproducing order with the stream pool off (the worst history seen), the whole
# GPU suite, smoke(), then the bench line. Stops at a failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 env DDMI_STREAM_POOL=0 python -u -m pytest tests/test_runner.py tests/test_inflight_gpu.py \
  tests/test_agent.py -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/order.log 2>&1
rc=$?; echo "[order] rc=$rc"; tail -1 gpurun_out/order.log; [ $rc -ne 0 ] && exit $rc
bash tools/archive/gpu_final_check.sh
