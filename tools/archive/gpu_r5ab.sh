#!/bin/bash
# round 5ab: tf-decoder megakernel at four workgroups per scene - parity tests, C1 A/B, bench A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_parity_gpu.py tests/test_ops_gpu.py -v -m gpu -x -rf --timeout 240 --timeout-method thread -k "tf_decoder or reference_goldens or deep_ring" > gpurun_out/r5ab_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; grep -E "passed|failed|Error|tf-decoder|max abs|waypoint" gpurun_out/r5ab_tests.log | tail -30; [ $rc -ne 0 ] && exit $rc
cat gpurun_out/parity_report.txt 2>/dev/null | grep -A7 "4 workgroups" | head -20
for cfg in "X=0" "DDMI_TF_GROUPS=1" "X=0" "DDMI_TF_GROUPS=1"; do
  env $cfg timeout -k 10 300 python -u tools/bench_configs.py --c1-child --c1-streams 2 --steps 20 > gpurun_out/r5ab_c1.log 2>&1
  rc=$?; echo "[c1 $cfg] rc=$rc $(grep C1TWO gpurun_out/r5ab_c1.log)"; [ $rc -ne 0 ] && exit $rc
done
TAG=r5ab REPS=2 bash tools/gpu_ab.sh "X=0" "DDMI_TF_GROUPS=1"
