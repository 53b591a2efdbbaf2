#!/bin/bash
# GPU-box check: per-op parity, then end-to-end parity. Stops at the first crash/timeout.
set -u
mkdir -p gpurun_out
run() {  # run <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[$name] abnormal exit ($rc): stopping"; exit $rc; fi
  return 0
}
run ops 600 python -m pytest tests/test_ops_gpu.py -q -m gpu -rf
run parity 900 python -m pytest tests/test_parity_gpu.py -q -m gpu -rf -s
