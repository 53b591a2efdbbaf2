#!/bin/bash
# Round-4 (f): the round-3 reproducing order with the dbg library and the stream pool off, output uncaptured (-s) so
# the library's SIGSEGV backtrace and lifecycle trace lines reach the log (a segfault is the expected finding).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 env DDMI_STREAM_POOL=0 DDMI_LIB=$R/diffusiondrive_amd/_variants/libddmi_dbg.so python -u -m pytest \
  tests/test_runner.py tests/test_inflight_gpu.py tests/test_agent.py -v -s -m gpu -x --timeout 300 --timeout-method thread \
  > gpurun_out/order_dbg_s.log 2>&1; rc=$?; echo "[order_dbg_s] rc=$rc"; grep -n -A40 "SIGSEGV" gpurun_out/order_dbg_s.log | head -60; exit $rc
