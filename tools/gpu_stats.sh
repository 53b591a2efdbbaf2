#!/bin/bash
# GPU box: rocprofv3 kernel stats of a short single-stream bench (per-instance average durations).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
DDMI_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/st" -o run -- python "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-compare > "$R/gpurun_out/st.log" 2>&1
rc=$?; echo "[stats] rc=$rc"; exit $rc
