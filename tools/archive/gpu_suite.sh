#!/bin/bash
# The round-end GPU checks: (1) the reproducing order with the stream pool off (the worst history
# seen); (2) the whole GPU suite in its default order (the driver's round-end run); (3) smoke(). Stops at a failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 env DDMI_STREAM_POOL=0 python -u -m pytest tests/test_runner.py tests/test_inflight_gpu.py \
  tests/test_agent.py -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/order_single_default.log 2>&1
rc=$?; echo "[order] rc=$rc"; tail -2 gpurun_out/order_single_default.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x -rf --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; echo "[suite] rc=$rc"; tail -3 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "[smoke] rc=$rc"; tail -2 gpurun_out/smoke.log; exit $rc
