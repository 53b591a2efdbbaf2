#!/bin/bash
# round 5ah: fused GPT block tail (C <= 128) - bit-identity / goldens / determinism tests, C1 A/B, bench A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -v -m gpu -x -rf --timeout 300 --timeout-method thread -k "gpt_tail or layernorm_fold or reference_goldens or deterministic_across" > gpurun_out/r5ah_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc $(tail -1 gpurun_out/r5ah_tests.log)"; grep -E "^E  .{0,200}|FAILED" -o gpurun_out/r5ah_tests.log | head -8; [ $rc -ne 0 ] && exit $rc
for cfg in "X=0" "DDMI_GPT_TAIL=0" "X=0" "DDMI_GPT_TAIL=0"; do
  env $cfg timeout -k 10 300 python -u tools/bench_configs.py --c1-child --c1-streams 2 --steps 20 > gpurun_out/r5ah_c1.log 2>&1
  rc=$?; echo "[c1 $cfg] rc=$rc $(grep C1TWO gpurun_out/r5ah_c1.log | cut -c1-80)"; [ $rc -ne 0 ] && exit $rc
done
TAG=r5ah REPS=2 bash tools/gpu_ab.sh "X=0" "DDMI_GPT_TAIL=0"
