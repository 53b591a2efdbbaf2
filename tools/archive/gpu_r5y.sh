#!/bin/bash
# round 5y: rocprofv3 kernel trace of the bench workload with single-stream handles (DDMI_STREAMS=0: every launch
# alone on the device, so its average duration compares with the bench's per-launch HIP events), then the PMC passes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
DDMI_STREAMS=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r5y_trace" -- python3 "$R/bench.py" --steps 5 --warmup 2 --in-flight 1 --no-cpu-baseline --no-compare > "$R/gpurun_out/r5y_trace.log" 2>&1
rc=$?; echo "[trace] rc=$rc"; tail -1 "$R/gpurun_out/r5y_trace.log" | cut -c1-200; [ $rc -ne 0 ] && exit $rc
cd "$R" && bash tools/gpu_pmc_round2.sh
