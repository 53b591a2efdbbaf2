#!/bin/bash
# round 5u: layer-1 convs at three workgroups per CU by default - tests, then bench A/B against the 16 x 16 form
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_ops_gpu.py tests/test_parity_gpu.py -v -m gpu -x --timeout 240 --timeout-method thread -k "three_per_cu or conv2d_f16x3_b64" > gpurun_out/r5u_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r5u_tests.log | tail -4; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for cfg in "X=0" "DDMI_X6_CFG=4"; do
    env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare --steps 100 > gpurun_out/r5u.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc [$cfg]"; tail -5 gpurun_out/r5u.log; exit $rc; }
    echo "[if3 $cfg] $(tail -1 gpurun_out/r5u.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["device_ms_per_step"]["conv_x6"], d["roofline"]["frac"])')"
    env $cfg timeout -k 10 300 python bench.py --in-flight 1 --no-cpu-baseline --no-compare --steps 200 > gpurun_out/r5u1.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc [$cfg]"; tail -5 gpurun_out/r5u1.log; exit $rc; }
    echo "[if1 $cfg] $(tail -1 gpurun_out/r5u1.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
  done
done | tee gpurun_out/r5u_ab.txt
