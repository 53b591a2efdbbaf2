#!/bin/bash
# round 5aq: conv_x3 K split ahead of conv_x6 at small grids (DDMI_X3_SPLIT=2) - parity, C1 A/B, batch-1 timeline
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
DDMI_X3_SPLIT=2 timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_ops_gpu.py -q -m gpu -x --timeout 300 --timeout-method thread -k "reference_goldens or boundary or k_split" > gpurun_out/r5aq_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc $(tail -1 gpurun_out/r5aq_tests.log)"; grep -E "^E  .{0,200}|FAILED" -o gpurun_out/r5aq_tests.log | head -6; [ $rc -ne 0 ] && exit $rc
for cfg in "DDMI_X3_SPLIT=2" "X=0" "DDMI_X3_SPLIT=2" "X=0"; do
  env $cfg timeout -k 10 300 python -u tools/bench_configs.py --c1-child --c1-streams 2 --steps 20 > gpurun_out/r5aq_c1.log 2>&1
  rc=$?; echo "[c1 $cfg] rc=$rc $(grep C1TWO gpurun_out/r5aq_c1.log | cut -c1-110)"; [ $rc -ne 0 ] && exit $rc
done
cd /tmp && export TMPDIR=/tmp
DDMI_X3_SPLIT=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/r5aq_b1" -- python3 "$R/tools/micro/b1_trace.py" > "$R/gpurun_out/r5aq_b1.log" 2>&1
rc=$?; echo "[trace] rc=$rc"; exit $rc
