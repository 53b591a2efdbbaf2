#!/bin/bash
# round-5 evidence on the final tree: C1, the reproducing order, the whole GPU suite, smoke, bench (tools/gpu_check.sh),
# then a rocprofv3 kernel trace of the bench workload (one batch at a time, summarised by tools/prof_summary.py)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
bash tools/gpu_check.sh r5z || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r5z_trace" -- python3 "$R/bench.py" --steps 10 --warmup 2 --in-flight 1 --no-cpu-baseline --no-compare > "$R/gpurun_out/r5z_trace.log" 2>&1
rc=$?; echo "[trace] rc=$rc"; tail -c 300 "$R/gpurun_out/r5z_trace.log"; exit $rc
