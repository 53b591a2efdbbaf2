#!/bin/bash
# One GPU call over the tree: C1 batch-1 latency (default two-stream handle, then single-stream; child processes),
# the reproducing order with the stream pool off, the whole GPU suite, smoke(), then the bench line.
# Usage (from the repo root): tools/gpu_check.sh [tag]   -> gpurun_out/<tag>_*.log
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
T=${1:-chk}
for ns in 2 1; do
  timeout -k 10 300 python -u tools/bench_configs.py --c1-child --c1-streams $ns --steps 20 > gpurun_out/${T}_c1_s$ns.log 2>&1
  rc=$?; echo "[c1 streams=$ns] rc=$rc"; grep C1TWO gpurun_out/${T}_c1_s$ns.log; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 env DDMI_STREAM_POOL=0 python -u -m pytest tests/test_runner.py tests/test_inflight_gpu.py \
  tests/test_agent.py -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/${T}_order.log 2>&1
rc=$?; echo "[order] rc=$rc"; tail -2 gpurun_out/${T}_order.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x -rf --durations=30 --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "[suite] rc=$rc"; tail -3 gpurun_out/${T}_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1
rc=$?; echo "[smoke] rc=$rc"; tail -2 gpurun_out/${T}_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.log 2>&1
rc=$?; echo "[bench] rc=$rc"; tail -c 600 gpurun_out/${T}_bench.log; exit $rc
