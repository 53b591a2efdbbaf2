#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_ops_gpu.py -q -m gpu -x -k "f16x3" > gpurun_out/x3_ops.log 2>&1
rc=$?; echo "[ops] rc=$rc"; tail -15 gpurun_out/x3_ops.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/launch_log.py --gemm f16x3 --out gpurun_out/launches_x3.md > gpurun_out/ll_x3.log 2>&1
rc=$?; echo "[ll] rc=$rc"; head -30 gpurun_out/launches_x3.md; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -m pytest tests/test_parity_gpu.py -q -m gpu -x > gpurun_out/x3_parity.log 2>&1
rc=$?; echo "[parity] rc=$rc"; tail -5 gpurun_out/x3_parity.log; exit $rc
