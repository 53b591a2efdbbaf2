#!/bin/bash
# round 6 (z): the tree's evidence run - C1, the reproducing order, the whole GPU suite, smoke, bench
# (tools/gpu_check.sh), then a rocprofv3 kernel trace of the bench workload with single-stream handles
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
T=${TAG:-r6z}
bash tools/gpu_check.sh $T || exit $?
cd /tmp && export TMPDIR=/tmp
DDMI_STREAMS=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${T}_trace" -- python3 "$R/bench.py" --steps 5 --warmup 2 --in-flight 1 --no-cpu-baseline --no-compare > "$R/gpurun_out/${T}_trace.log" 2>&1
rc=$?; echo "[trace] rc=$rc"; tail -c 300 "$R/gpurun_out/${T}_trace.log"; exit $rc
