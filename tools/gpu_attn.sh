#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -q -m gpu -x -rf -k "attention or softmax" --timeout 120 --timeout-method thread > gpurun_out/tests_attn.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -2 gpurun_out/tests_attn.log; [ $rc -ne 0 ] && exit $rc
for d in ${DBGS:-0}; do
  echo "== DDMI_ATT_DBG=$d"
  DDMI_ATT_DBG=$d timeout -k 10 120 python tools/micro/attn_bench.py > gpurun_out/attn_$d.log 2>&1
  rc=$?; cat gpurun_out/attn_$d.log | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
done
exit 0
