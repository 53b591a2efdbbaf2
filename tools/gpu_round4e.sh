#!/bin/bash
# Round-4 (e): the two-per-CU conv_x6 form (DDMI_X6_CFG=3) against the op tests / goldens, per-shape and bench A/B;
# the training-head GPU tests; then the handle-lifetime investigation: the minimal reproducer with every stream of
# the process re-created per iteration, and the round-3 reproducing order with the dbg library and the pool off
# (a segfault in either is the finding: nothing runs after it).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 env DDMI_X6_CFG=3 python -u -m pytest tests/test_ops_gpu.py tests/test_parity_gpu.py -m gpu -x -q \
  -k "conv or golden or value_proj" --timeout 300 --timeout-method thread > gpurun_out/cfg3_test.log 2>&1; rc=$?
tail -3 gpurun_out/cfg3_test.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/x6cfg3.log; : > $out
for shp in img.l2.3x3 img.l3.3x3 img.l4.3x3 lid.l2.3x3 lid.l3.3x3; do
  for v in "DDMI_X6_CFG=0" "DDMI_X6_CFG=3" "DDMI_X6_CFG=0"; do
    r=$(env $v timeout -k 5 60 tools/micro/conv_bench 20 $shp 2>&1 | tail -1); rc=$?
    [ $rc -ne 0 ] && { echo "rc=$rc $shp $v"; exit $rc; }
    echo "[$v] $r" | tee -a $out
  done
done
STEPS=60 bash tools/gpu_envab.sh "DDMI_NONE=0" "DDMI_X6_CFG=3" | tee gpurun_out/envab_cfg3.txt || exit $?
timeout -k 10 300 python -u -m pytest tests/test_train_loss.py -v -m gpu -x --timeout 200 --timeout-method thread \
  > gpurun_out/train_tests.log 2>&1; rc=$?; tail -3 gpurun_out/train_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 tools/repro/graph_churn 150 0 64 1 > gpurun_out/churn_all.log 2>&1; rc=$?
echo "[churn_all] rc=$rc"; tail -2 gpurun_out/churn_all.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 env DDMI_STREAM_POOL=0 DDMI_LIB=$R/diffusiondrive_amd/_variants/libddmi_dbg.so python -u -m pytest \
  tests/test_runner.py tests/test_inflight_gpu.py tests/test_agent.py -v -m gpu -x --timeout 300 --timeout-method thread \
  > gpurun_out/order_dbg.log 2>&1; rc=$?; echo "[order_dbg] rc=$rc"; tail -3 gpurun_out/order_dbg.log; exit $rc
