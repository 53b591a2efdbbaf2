#!/bin/bash
# Round-4 (d): round4c's experiments, the training-head GPU tests, then (last: a segfault there is the finding) the
# handle-lifetime investigation with the dbg library in the round-3 reproducing order with the stream pool off.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
STEPS=60 bash tools/gpu_round4c.sh || exit $?
timeout -k 10 300 python -u -m pytest tests/test_train_loss.py -v -m gpu -x --timeout 200 --timeout-method thread \
  > gpurun_out/train_tests.log 2>&1; rc=$?; tail -3 gpurun_out/train_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 env DDMI_STREAM_POOL=0 DDMI_LIB=$R/diffusiondrive_amd/_variants/libddmi_dbg.so python -u -m pytest \
  tests/test_runner.py tests/test_inflight_gpu.py tests/test_agent.py -v -m gpu -x --timeout 300 --timeout-method thread \
  > gpurun_out/order_dbg.log 2>&1; rc=$?; echo "[order_dbg] rc=$rc"; tail -3 gpurun_out/order_dbg.log; exit $rc
