#!/bin/bash
# round 5e: value_proj split reduction (coalesced, <= 8 splits) + conv_x6 two-per-CU BN = 128 form (DDMI_X6_CFG=3):
# tests, B = 1 latency and trace, conv micro-benchmark A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_ops_gpu.py -v -m gpu -x --timeout 240 --timeout-method thread -k "value_proj_variants or two_per_cu or conv2d_f16x3_b64 or forward_matches_reference_goldens or stem_pool or nchw_stem" > gpurun_out/r5e_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; grep -E "passed|failed|Error|max err" gpurun_out/r5e_tests.log | tail -8; grep -E "union_split|trajectory" gpurun_out/parity_report.txt | tail -12; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/bench_configs.py --c1-child --c1-streams 2 --steps 20 > gpurun_out/r5e_c1.log 2>&1
rc=$?; echo "[c1] rc=$rc"; grep C1TWO gpurun_out/r5e_c1.log; [ $rc -ne 0 ] && exit $rc
for shp in img.l2.3x3 img.l3.3x3 lid.l2.3x3 lid.l3.3x3 fx.l3.c128; do
  for cfg in "DDMI_X6_CFG=0" "DDMI_X6_CFG=3"; do
    out=$(env $cfg timeout -k 5 60 tools/micro/conv_bench ${REPS:-30} $shp 2>&1)
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc $shp [$cfg]"; echo "$out"; exit $rc; }
    echo "$out" | awk -v s="$shp" -v c="[$cfg]" '$1 == s { print c " " $0 }'
  done
done > gpurun_out/r5e_convab.txt
rc=$?; cat gpurun_out/r5e_convab.txt; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/r5e_b1trace" -- python3 "$R/tools/micro/b1_trace.py" > "$R/gpurun_out/r5e_b1trace.log" 2>&1
rc=$?; echo "[b1 trace] rc=$rc"; grep b1_trace "$R/gpurun_out/r5e_b1trace.log"; exit $rc
