#!/bin/bash
# HBM traffic per kernel from two separate rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE cannot
# share a pass on gfx950; MI355X_MICROARCH.md "rocprofv3 PMC slots"), each with the kernel trace
# only. Summarise afterwards on the build container:
#   python tools/prof_summary.py gpurun_out/pmc_trace <name> --pmc gpurun_out/pmc_fetch gpurun_out/pmc_write
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps ${PMC_STEPS:-2} --warmup 1 --no-cpu-baseline --no-compare ${BENCH_ARGS:-}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/pmc_trace" -o run -- python "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_trace.log" 2>&1
rc=$?; echo "[trace] rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -f csv -d "$R/gpurun_out/pmc_fetch" -o run -- python "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_fetch.log" 2>&1
rc=$?; echo "[fetch] rc=$rc"; tail -2 "$R/gpurun_out/pmc_fetch.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -f csv -d "$R/gpurun_out/pmc_write" -o run -- python "$R/bench.py" $ARGS > "$R/gpurun_out/pmc_write.log" 2>&1
rc=$?; echo "[write] rc=$rc"; tail -2 "$R/gpurun_out/pmc_write.log"; exit $rc
