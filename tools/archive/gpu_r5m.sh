#!/bin/bash
# round 5m: union value_proj with a step barrier at every other step (BAR2) - variants test, stamps, A/B on the bench
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -v -m gpu -x --timeout 300 --timeout-method thread -k "value_proj_variants or forward_matches_reference_goldens" > gpurun_out/r5m_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r5m_tests.log | tail -4; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python -u tools/micro/vu_stamps.py > gpurun_out/r5m_vu_stamps.txt 2>&1
rc=$?; tail -2 gpurun_out/r5m_vu_stamps.txt; [ $rc -ne 0 ] && exit $rc
DDMI_VPROJ_BAR=1 timeout -k 10 240 python -u tools/micro/vu_stamps.py > gpurun_out/r5m_vu_stamps_bar1.txt 2>&1
rc=$?; tail -2 gpurun_out/r5m_vu_stamps_bar1.txt; [ $rc -ne 0 ] && exit $rc
for cfg in "X=0" "DDMI_VPROJ_BAR=1" "X=0" "DDMI_VPROJ_BAR=1"; do
  env $cfg timeout -k 10 200 python bench.py --in-flight 1 --no-cpu-baseline --no-compare --steps 40 > gpurun_out/r5m.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc [$cfg]"; tail -5 gpurun_out/r5m.log; exit $rc; }
  echo "[if1 $cfg] $(tail -1 gpurun_out/r5m.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["device_ms_per_step"]["value_proj"], d["decoder_cross_attention"]["avg_launch_ms"])')"
done | tee gpurun_out/r5m_ab.txt
