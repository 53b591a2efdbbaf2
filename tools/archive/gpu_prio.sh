#!/bin/bash
# Two-stream graphs launched from a greatest-priority stream (DDMI_MAIN_PRIORITY=1): (1) the reproducing order with
# two-stream graphs and the stream pool off (faulted 6 of 6 without the priority); (2) the runtime's queue log of one
# such handle; (3) the whole GPU suite with two-stream graphs (faulted at test_train_loss without the priority);
# (4) one-at-a-time bench A/B (fresh processes). Stops at a failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
P="DDMI_STREAMS=1 DDMI_MAIN_PRIORITY=1"
timeout -k 10 400 env DDMI_STREAM_POOL=0 $P python -u -m pytest tests/test_runner.py tests/test_inflight_gpu.py \
  tests/test_agent.py -v -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/prio_order.log 2>&1
rc=$?; echo "[prio order] rc=$rc"; tail -2 gpurun_out/prio_order.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 env $P AMD_LOG_LEVEL=3 python tools/repro/handle_churn.py 2 0 1 0 > /tmp/prio_log.txt 2>&1
rc=$?; echo "[prio log] rc=$rc"; grep -a "Number of allocated hardware queues\|Selected queue\|hipGraphInstantiate (\|hipStreamCreateWithPriority (" /tmp/prio_log.txt | sed 's/\x1b\[[0-9;]*m//g' | head -60 > gpurun_out/prio_queues.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 env $P python -u -m pytest tests -v -m gpu -x -rf --timeout 300 --timeout-method thread > gpurun_out/prio_suite.log 2>&1
rc=$?; echo "[prio suite] rc=$rc"; tail -2 gpurun_out/prio_suite.log; [ $rc -ne 0 ] && exit $rc
STEPS=60 BENCH_EXTRA="--in-flight 1" bash tools/archive/gpu_envab.sh "DDMI_NONE=0" "DDMI_STREAMS=1 DDMI_MAIN_PRIORITY=1" "DDMI_STREAMS=1" | tee gpurun_out/prio_envab.txt
