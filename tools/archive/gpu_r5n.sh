#!/bin/bash
# round 5n: layer 1 in MALL-sized scene chunks (DDMI_S0_CHUNK_MB, default 72; 0 = whole batch) - goldens, bit-identity
# against the whole-batch stage, A/B on the bench (one at a time, 3 in flight), same box
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -v -m gpu -x --timeout 300 --timeout-method thread -k "forward_matches_reference_goldens or stage_chunk" > gpurun_out/r5n_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; grep -E "passed|failed|Error" gpurun_out/r5n_tests.log | tail -4; [ $rc -ne 0 ] && exit $rc
for cfg in "X=0" "DDMI_S0_CHUNK_MB=0" "X=0" "DDMI_S0_CHUNK_MB=0"; do
  env $cfg timeout -k 10 200 python bench.py --in-flight 1 --no-cpu-baseline --no-compare --steps 40 > gpurun_out/r5n.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc [$cfg]"; tail -5 gpurun_out/r5n.log; exit $rc; }
  echo "[if1 $cfg] $(tail -1 gpurun_out/r5n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["device_ms_per_step"]["conv_x6"], d["launches_per_step"]["conv_x6"])')"
done | tee gpurun_out/r5n_ab.txt
for cfg in "X=0" "DDMI_S0_CHUNK_MB=0" "X=0" "DDMI_S0_CHUNK_MB=0"; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --no-compare --steps 100 > gpurun_out/r5n3.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc [$cfg]"; tail -5 gpurun_out/r5n3.log; exit $rc; }
  echo "[if3 $cfg] $(tail -1 gpurun_out/r5n3.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
done | tee -a gpurun_out/r5n_ab.txt
