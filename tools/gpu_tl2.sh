#!/bin/bash
# GPU box: full gpu tests, bench, then a two-stream kernel trace for tools/timeline.py. Stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -rf --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "[bench] rc=$rc"; cut -c1-260 gpurun_out/bench.json; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d "$R/gpurun_out/tl" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-compare > "$R/gpurun_out/tl.log" 2>&1
rc=$?; echo "[trace] rc=$rc"; exit $rc
