#!/bin/bash
# The round-4 handle-lifetime investigation (profiles/round4_f_handle_lifetime.md) as one script:
#   tools/archive/gpu_handle_lifetime.sh <step> [env ...]
# steps:
#   order   the reproducing order (test_runner -> test_inflight_gpu -> test_agent), stream pool off; extra env applies
#           (e.g. DDMI_STREAMS=1 to run it with the two-stream graphs that faulted)
#   amdlog  the same with the HIP runtime's info log (AMD_LOG_LEVEL=3) to /tmp; only its tail comes back
#   churn   the pure-HIP reproducer (tools/repro/graph_churn) and the library-only churn (tools/repro/handle_churn.py)
#   asan    host AddressSanitizer over the library's host code (tools/repro/asan_driver; build: tools/repro/build_asan.sh)
# One step per GPU call: a segfault ends the call.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
step=${1:-order}; shift || true
ORDER="tests/test_runner.py tests/test_inflight_gpu.py tests/test_agent.py"
case $step in
  order)
    timeout -k 10 400 env DDMI_STREAM_POOL=0 "$@" python -u -m pytest $ORDER -v -m gpu -x --timeout 300 \
      --timeout-method thread > gpurun_out/order.log 2>&1
    rc=$?; echo "[order] rc=$rc"; tail -2 gpurun_out/order.log; exit $rc ;;
  amdlog)
    timeout -k 10 500 env DDMI_STREAM_POOL=0 AMD_LOG_LEVEL=3 "$@" python -u -m pytest $ORDER -v -s -m gpu -x \
      --timeout 400 --timeout-method thread > /tmp/amdlog.txt 2>&1
    rc=$?; echo "[amdlog] rc=$rc"
    grep -n "Selected queue\|releaseQueue\|hipStreamCreate\|hipStreamDestroy\|hipGraphInstantiate\|hipGraphLaunch" \
      /tmp/amdlog.txt | tail -400 > gpurun_out/amdlog_queues.txt
    tail -c 12000000 /tmp/amdlog.txt > gpurun_out/amdlog_tail.txt; exit $rc ;;
  churn)
    for a in "150 0 64 1" "60 0 512 0 4 1"; do
      timeout -k 10 300 tools/repro/graph_churn $a > gpurun_out/churn.log 2>&1; rc=$?
      echo "[graph_churn $a] rc=$rc"; tail -1 gpurun_out/churn.log; [ $rc -ne 0 ] && exit $rc
    done
    timeout -k 10 600 env DDMI_STREAM_POOL=0 "$@" python -u tools/repro/handle_churn.py 50 0 1 1 > gpurun_out/hchurn.log 2>&1
    rc=$?; echo "[handle_churn] rc=$rc"; tail -2 gpurun_out/hchurn.log; exit $rc ;;
  asan)
    python -c "from diffusiondrive_amd.config import TransfuserConfig as C; from diffusiondrive_amd.weights import \
seeded_state_dict as s, pack_blob as p; open('/tmp/dd_w.ddw1', 'wb').write(p(s(C(), 0)))" || exit 1
    timeout -k 10 900 env ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0:halt_on_error=1 tools/repro/asan_driver \
      /tmp/dd_w.ddw1 45 > gpurun_out/asan.log 2>&1
    rc=$?; echo "[asan] rc=$rc"; tail -2 gpurun_out/asan.log; exit $rc ;;
  *) echo "unknown step $step"; exit 2 ;;
esac
