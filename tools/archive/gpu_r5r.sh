#!/bin/bash
# round 5r: conv_x6 small-grid form (8 x 8 x 64) - op tests, goldens, C1 batch-1 latency with and without, B = 1 trace
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_parity_gpu.py -v -m gpu -x --timeout 240 --timeout-method thread -k "small_grid or conv2d_f16x3 or conv2d_bf16 or forward_matches_reference_goldens" > gpurun_out/r5r_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; grep -E "passed|failed|Error|max err" gpurun_out/r5r_tests.log | tail -6; [ $rc -ne 0 ] && exit $rc
for cfg in "X=0" "DDMI_X6_SMALL=0" "X=0" "DDMI_X6_SMALL=0"; do
  env $cfg timeout -k 10 300 python -u tools/bench_configs.py --c1-child --c1-streams 2 --steps 20 > gpurun_out/r5r_c1.log 2>&1
  rc=$?; echo "[c1 $cfg] rc=$rc $(grep C1TWO gpurun_out/r5r_c1.log)"; [ $rc -ne 0 ] && exit $rc
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/r5r_b1trace" -- python3 "$R/tools/micro/b1_trace.py" > "$R/gpurun_out/r5r_b1trace.log" 2>&1
rc=$?; echo "[b1 trace] rc=$rc"; grep b1_trace "$R/gpurun_out/r5r_b1trace.log"; exit $rc
