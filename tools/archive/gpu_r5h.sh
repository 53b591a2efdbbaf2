#!/bin/bash
# round 5h: goldens + decoder query groups (now capped at B x G <= 64), bench, PMC passes over the bench workload
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -v -m gpu -x --timeout 240 --timeout-method thread -k "forward_matches_reference_goldens or decoder_query_groups" > gpurun_out/r5h_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r5h_tests.log | tail -4; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/r5h_bench.log 2>&1
rc=$?; echo "[bench] rc=$rc"; tail -1 gpurun_out/r5h_bench.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_pmc_round2.sh
