#!/bin/bash
# Round-end evidence (the GPU suite and smoke: tools/archive/gpu_suite.sh): the bench line, the rocprofv3 kernel
# trace of the bench workload (single stream, in flight 1), then the PMC passes (tools/gpu_pmc_round2.sh).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "[bench] rc=$rc"; tail -c 600 gpurun_out/bench.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/prof" -o run -- python "$R/bench.py" \
  --steps 5 --warmup 2 --no-cpu-baseline --no-compare --in-flight 1 > "$R/gpurun_out/prof.log" 2>&1
rc=$?; echo "[rocprof] rc=$rc"; tail -2 "$R/gpurun_out/prof.log"; [ $rc -ne 0 ] && exit $rc
cd "$R" && bash tools/gpu_pmc_round2.sh
