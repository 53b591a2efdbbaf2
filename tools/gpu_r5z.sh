#!/bin/bash
# round-5 evidence on the final tree: C1, the reproducing order, the whole GPU suite, smoke, bench (tools/gpu_check.sh),
# then a rocprofv3 kernel trace of the bench workload with single-stream handles (summarised by tools/prof_summary.py)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
bash tools/gpu_check.sh ${TAG:-r5z} || exit $?
cd /tmp && export TMPDIR=/tmp
DDMI_STREAMS=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${TAG:-r5z}_trace" -- python3 "$R/bench.py" --steps 5 --warmup 2 --in-flight 1 --no-cpu-baseline --no-compare > "$R/gpurun_out/${TAG:-r5z}_trace.log" 2>&1
rc=$?; echo "[trace] rc=$rc"; tail -c 300 "$R/gpurun_out/${TAG:-r5z}_trace.log"; exit $rc
