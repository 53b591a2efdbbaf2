#!/bin/bash
# Round-3 GPU session: a parity subset (TESTK), the bench, then the per-kernel-class PMC passes of
# tools/gpu_pmc_round2.sh (MFMA busy, LDS, FETCH, WRITE, L2). Stops at the first abnormal exit.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "${TESTK:-gathered or compacted or golden or boundary}" \
  --timeout 300 --timeout-method thread > gpurun_out/tests3.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/tests3.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench3.log 2>&1
rc=$?; echo "[bench] rc=$rc"; tail -1 gpurun_out/bench3.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
[ "${PMC:-1}" = "1" ] || exit 0
bash tools/gpu_pmc_round2.sh
