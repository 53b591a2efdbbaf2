#!/bin/bash
# round 5at: the K-split reduce with all splits' loads hoisted (template S) vs the runtime-S loop - parity, C1 A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_parity_gpu.py -q -m gpu -x --timeout 300 --timeout-method thread -k "k_split or reference_goldens or boundary or deterministic" > gpurun_out/r5at_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc $(tail -1 gpurun_out/r5at_tests.log)"; grep -E "^E  .{0,200}|FAILED" -o gpurun_out/r5at_tests.log | head -6; [ $rc -ne 0 ] && exit $rc
for cfg in "X=0" "DDMI_X3_RED_LOOP=1" "X=0" "DDMI_X3_RED_LOOP=1"; do
  env $cfg timeout -k 10 300 python -u tools/bench_configs.py --c1-child --c1-streams 2 --steps 20 > gpurun_out/r5at_c1.log 2>&1
  rc=$?; echo "[c1 $cfg] rc=$rc $(grep C1TWO gpurun_out/r5at_c1.log | cut -c1-110)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
