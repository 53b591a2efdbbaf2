#!/bin/bash
# Round-4 (c): value_proj N-half form parity, conv_x6 activation cache-policy sweep (micro-benchmark), then same-box
# bench A/B of the new knobs at 3 batches in flight and one at a time.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -v -m gpu -x -k "value_proj_variants" --timeout 300 \
  --timeout-method thread > gpurun_out/vp_test.log 2>&1; rc=$?; tail -3 gpurun_out/vp_test.log; [ $rc -ne 0 ] && exit $rc
# the relaxed conv_x6 barrier against the goldens and the op tests before it is timed
timeout -k 10 400 env DDMI_X6_RELAX=1 python -u -m pytest tests/test_ops_gpu.py tests/test_parity_gpu.py -m gpu -x -q \
  -k "conv or golden" --timeout 300 --timeout-method thread > gpurun_out/relax_test.log 2>&1; rc=$?
tail -3 gpurun_out/relax_test.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 env DDMI_X6_CFG=3 python -u -m pytest tests/test_ops_gpu.py tests/test_parity_gpu.py -m gpu -x -q \
  -k "conv or golden" --timeout 300 --timeout-method thread > gpurun_out/cfg3_test.log 2>&1; rc=$?
tail -3 gpurun_out/cfg3_test.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_x6nt.sh || exit $?
bash tools/gpu_envab.sh "DDMI_NONE=0" "DDMI_VPROJ_N=2" "DDMI_X6_NT=1" "DDMI_X6_RELAX=1" "DDMI_X6_CFG=3" | tee gpurun_out/envab_if3.txt || exit $?
BENCH_EXTRA="--in-flight 1" bash tools/gpu_envab.sh "DDMI_NONE=0" "DDMI_VPROJ_N=2" "DDMI_X6_RELAX=1" "DDMI_X6_CFG=3" | tee gpurun_out/envab_if1.txt || exit $?
