#!/bin/bash
# GPU box: gpu tests, then the per-launch breakdown (tools/launch_log.py). Stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -rf --timeout 300 --timeout-method thread ${TESTS:-} > gpurun_out/tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -4 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/launch_log.py --gemm f16x3 --out gpurun_out/ll.md > gpurun_out/ll.log 2>&1
rc=$?; echo "[ll] rc=$rc"; head -1 gpurun_out/ll.md; grep -A30 "GEMM / conv total" gpurun_out/ll.md; exit $rc
