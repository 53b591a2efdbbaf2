#!/bin/bash
# GPU box: rocprofv3 kernel trace of the bench (graph replays, no CPU baseline / comparison leg).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/trace" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-compare ${BENCH_ARGS:-} > "$R/gpurun_out/trace.log" 2>&1
rc=$?; echo "[trace] rc=$rc"; tail -2 "$R/gpurun_out/trace.log"; exit $rc
