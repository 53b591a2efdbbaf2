#!/bin/bash
# round 5h: stem fragment-read pipelining (goldens + stem tests, stem timing), C1 latency, bench, PMC passes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
bash tools/gpu_r5g.sh || exit $?
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/r5h_bench.log 2>&1
rc=$?; echo "[bench] rc=$rc"; tail -1 gpurun_out/r5h_bench.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_pmc_round2.sh
