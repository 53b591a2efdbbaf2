#!/bin/bash
# Round-4 (k): the reproducing order (runner -> inflight -> the agent's compute_trajectory, stream pool off) with the
# HIP runtime's info log (AMD_LOG_LEVEL=3: API calls, queue / resource messages) to a scratch file; only its tail comes
# back. The segfault is the expected end of the GPU step; the tail copy after it touches no GPU.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 500 env DDMI_STREAM_POOL=0 AMD_LOG_LEVEL=3 python -u -m pytest tests/test_runner.py \
  tests/test_inflight_gpu.py tests/test_agent.py::test_compute_trajectory_matches_oracle -v -s -m gpu -x \
  --timeout 400 --timeout-method thread > /tmp/amdlog.txt 2>&1
rc=$?; echo "[order_amdlog] rc=$rc"; ls -la /tmp/amdlog.txt
grep -n "Deleting hardware queue\|acquireQueue\|releaseQueue\|Number of allocated hardware queues" /tmp/amdlog.txt | tail -400 > gpurun_out/amdlog_queues.txt
tail -c 12000000 /tmp/amdlog.txt > gpurun_out/amdlog_tail.txt
exit $rc
