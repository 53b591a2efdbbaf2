#!/bin/bash
# One-channel LiDAR stem (K = 64) against the 4-channel layout (DDMI_STEM1=0): parity tests, then bench A/B (same box).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_sharding_gpu.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/stem1_parity.log 2>&1
rc=$?; echo "[parity] rc=$rc"; tail -2 gpurun_out/stem1_parity.log; [ $rc -ne 0 ] && exit $rc
STEPS=100 bash tools/gpu_envab.sh "DDMI_STEM1=1" "DDMI_STEM1=0" "DDMI_STEM1=1" "DDMI_STEM1=0" | tee gpurun_out/stem1_envab.txt
