#!/bin/bash
# round 5t: conv_x6 layer-1 form at three workgroups per CU (8 x 16 tiles, DDMI_X6_CFG=4) - bit-identity test, A/B
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -v -m gpu -x --timeout 120 --timeout-method thread -k "three_per_cu" > gpurun_out/r5t_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r5t_tests.log | tail -4; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
for shp in img.l1.3x3 lid.l1.3x3; do
  for cfg in "DDMI_X6_CFG=0" "DDMI_X6_CFG=4"; do
    out=$(env $cfg timeout -k 5 60 tools/micro/conv_bench ${REPS:-30} $shp 2>&1)
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc $shp [$cfg]"; echo "$out"; exit $rc; }
    echo "$out" | awk -v s="$shp" -v c="[$cfg]" '$1 == s { print c " " $0 }'
  done
done
done > gpurun_out/r5t_ab.txt
rc=$?; cat gpurun_out/r5t_ab.txt; exit $rc
