#!/bin/bash
# round 5ao: fork / join events with a device-scope release - tests, C1 A/B, bench A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_parity_gpu.py tests/test_inflight_gpu.py -q -m gpu -x --timeout 300 --timeout-method thread -k "reference_goldens or deterministic or inflight or groups_match" > gpurun_out/r5ao_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc $(tail -1 gpurun_out/r5ao_tests.log)"; [ $rc -ne 0 ] && exit $rc
for cfg in "X=0" "DDMI_FJ_SYSTEM=1" "X=0" "DDMI_FJ_SYSTEM=1"; do
  env $cfg timeout -k 10 300 python -u tools/bench_configs.py --c1-child --c1-streams 2 --steps 20 > gpurun_out/r5ao_c1.log 2>&1
  rc=$?; echo "[c1 $cfg] rc=$rc $(grep C1TWO gpurun_out/r5ao_c1.log | cut -c1-80)"; [ $rc -ne 0 ] && exit $rc
done
TAG=r5ao REPS=2 bash tools/gpu_ab.sh "X=0" "DDMI_FJ_SYSTEM=1"
