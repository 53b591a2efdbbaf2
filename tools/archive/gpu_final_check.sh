#!/bin/bash
# Final tree: the whole GPU suite (default order, default configuration), smoke(), then the bench line.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x -rf --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; echo "[suite] rc=$rc"; tail -2 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "[smoke] rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "[bench] rc=$rc"; tail -c 300 gpurun_out/bench.log; exit $rc
