#!/bin/bash
# GPU box: gpu tests then one bench line (no CPU baseline). Stops at the first abnormal exit.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -rf --timeout 300 --timeout-method thread ${TESTS:-} > gpurun_out/tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -4 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "[bench] rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err; exit $rc
