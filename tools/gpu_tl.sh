#!/bin/bash
# GPU box: one two-stream kernel trace of the default bench graph (read with tools/tail_view.py gpurun_out/tl).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d "$R/gpurun_out/tl" -o run -- python "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-compare > "$R/gpurun_out/tl.log" 2>&1
rc=$?; echo "[trace] rc=$rc"; grep '^{' "$R/gpurun_out/tl.log" | cut -c1-150; exit $rc
