#!/bin/bash
# round 5al: fork events recorded inside the main segment (DDMI_SEG_FORK=1) - tests, C1, bench A/B against the default
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
DDMI_SEG_FORK=1 timeout -k 10 700 python -u -m pytest tests/test_parity_gpu.py tests/test_inflight_gpu.py tests/test_boundary_gpu.py -q -m gpu -x --timeout 300 --timeout-method thread -k "reference_goldens or deterministic or inflight or multi_stream or graph" > gpurun_out/r5al_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc $(tail -1 gpurun_out/r5al_tests.log)"; grep -E "^E  .{0,200}|FAILED" -o gpurun_out/r5al_tests.log | head -6; [ $rc -ne 0 ] && exit $rc
for cfg in "DDMI_SEG_FORK=1" "X=0" "DDMI_SEG_FORK=1" "X=0"; do
  env $cfg timeout -k 10 300 python -u tools/bench_configs.py --c1-child --c1-streams 2 --steps 20 > gpurun_out/r5al_c1.log 2>&1
  rc=$?; echo "[c1 $cfg] rc=$rc $(grep C1TWO gpurun_out/r5al_c1.log | cut -c1-80)"; [ $rc -ne 0 ] && exit $rc
done
TAG=r5al REPS=2 bash tools/gpu_ab.sh "DDMI_SEG_FORK=1" "X=0"
