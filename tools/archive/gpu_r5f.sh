#!/bin/bash
# round 5f: tests of this round's changes, B = 1 latency, conv_x6 two-per-CU A/B, stem phase split (DDMI_STEM_DIAG) and
# the one-channel LiDAR form's time (DDMI_STEM1), B = 1 trace
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_ops_gpu.py -v -m gpu -x --timeout 240 --timeout-method thread -k "two_per_cu or stem_pool" > gpurun_out/r5f_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; grep -E "passed|failed|Error|max err" gpurun_out/r5f_tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/bench_configs.py --c1-child --c1-streams 2 --steps 20 > gpurun_out/r5f_c1.log 2>&1
rc=$?; echo "[c1] rc=$rc"; grep C1TWO gpurun_out/r5f_c1.log; [ $rc -ne 0 ] && exit $rc
for shp in img.l2.3x3 img.l3.3x3 lid.l2.3x3 lid.l3.3x3 fx.l3.c128; do
  for cfg in "DDMI_X6_CFG=0" "DDMI_X6_CFG=3"; do
    out=$(env $cfg timeout -k 5 60 tools/micro/conv_bench ${REPS:-30} $shp 2>&1)
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc $shp [$cfg]"; echo "$out"; exit $rc; }
    echo "$out" | awk -v s="$shp" -v c="[$cfg]" '$1 == s { print c " " $0 }'
  done
done > gpurun_out/r5f_convab.txt
rc=$?; cat gpurun_out/r5f_convab.txt; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for v in "0 0" "1 0" "2 0" "3 0" "0 1"; do
  set -- $v
  DDMI_STEM_DIAG=$1 DDMI_STEM1=$2 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r5f_stem_d$1_o$2" -- python3 "$R/tools/micro/stem_time.py" > "$R/gpurun_out/r5f_stem_d$1_o$2.log" 2>&1
  rc=$?; echo "[stem diag=$1 one=$2] rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/r5f_b1trace" -- python3 "$R/tools/micro/b1_trace.py" > "$R/gpurun_out/r5f_b1trace.log" 2>&1
rc=$?; echo "[b1 trace] rc=$rc"; grep b1_trace "$R/gpurun_out/r5f_b1trace.log"; exit $rc
