#!/bin/bash
# stream of the process re-created per iteration, and the round-3 reproducing order with the dbg library and the pool
# off (a segfault in either is the finding: nothing runs after it).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_train_loss.py -v -m gpu -x --timeout 200 --timeout-method thread \
  > gpurun_out/train_tests.log 2>&1; rc=$?; tail -3 gpurun_out/train_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 tools/repro/graph_churn 150 0 64 1 > gpurun_out/churn_all.log 2>&1; rc=$?
echo "[churn_all] rc=$rc"; tail -2 gpurun_out/churn_all.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 env DDMI_STREAM_POOL=0 DDMI_LIB=$R/diffusiondrive_amd/_variants/libddmi_dbg.so python -u -m pytest \
  tests/test_runner.py tests/test_inflight_gpu.py tests/test_agent.py -v -m gpu -x --timeout 300 --timeout-method thread \
  > gpurun_out/order_dbg.log 2>&1; rc=$?; echo "[order_dbg] rc=$rc"; tail -3 gpurun_out/order_dbg.log; exit $rc
