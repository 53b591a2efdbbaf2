#!/bin/bash
# round 5as: conv_x3 K split with the last split reducing in-kernel (DDMI_X3_SPLIT_FUSE=1) - parity, C1 A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -q -m gpu -x --timeout 120 --timeout-method thread -k "k_split" > gpurun_out/r5ar_ops.log 2>&1
rc=$?; echo "[ops] rc=$rc $(tail -1 gpurun_out/r5ar_ops.log)"; grep -E "^E  .{0,200}|FAILED" -o gpurun_out/r5ar_ops.log | head -6; [ $rc -ne 0 ] && exit $rc
DDMI_X3_SPLIT_FUSE=1 timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_inflight_gpu.py -q -m gpu -x --timeout 300 --timeout-method thread -k "reference_goldens or deterministic or boundary or inflight" > gpurun_out/r5ar_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc $(tail -1 gpurun_out/r5ar_tests.log)"; grep -E "^E  .{0,200}|FAILED" -o gpurun_out/r5ar_tests.log | head -6; [ $rc -ne 0 ] && exit $rc
for cfg in "DDMI_X3_SPLIT_FUSE=1" "X=0" "DDMI_X3_SPLIT_FUSE=1" "X=0"; do
  env $cfg timeout -k 10 300 python -u tools/bench_configs.py --c1-child --c1-streams 2 --steps 20 > gpurun_out/r5ar_c1.log 2>&1
  rc=$?; echo "[c1 $cfg] rc=$rc $(grep C1TWO gpurun_out/r5ar_c1.log | cut -c1-110)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
