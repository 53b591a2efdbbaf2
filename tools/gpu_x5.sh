#!/bin/bash
# GPU box: conv op tests, then per-shape launch breakdown of the f16x3 forward and the bench. Stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -q -m gpu -x -rf --timeout 300 --timeout-method thread -k "conv or gemm" > gpurun_out/tests_ops.log 2>&1
rc=$?; echo "[ops] rc=$rc"; tail -3 gpurun_out/tests_ops.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/launch_log.py --gemm f16x3 --out gpurun_out/launches_f16x3.md > gpurun_out/ll.log 2>&1
rc=$?; echo "[ll] rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "[bench] rc=$rc"; cut -c1-300 gpurun_out/bench.json; exit $rc
