#!/bin/bash
# GPU-box bench + rocprofv3 kernel-trace summary. Stops at the first abnormal exit.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
timeout -k 10 600 python "$R/bench.py" "$@" > "$R/gpurun_out/bench.json" 2> "$R/gpurun_out/bench.err"
rc=$?; echo "[bench] rc=$rc"; cat "$R/gpurun_out/bench.json"; tail -3 "$R/gpurun_out/bench.err"
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run -- python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/prof.log" 2>&1
rc=$?; echo "[rocprof] rc=$rc"; tail -3 "$R/gpurun_out/prof.log"
exit $rc
