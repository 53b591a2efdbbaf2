#!/bin/bash
# round 5g: stem fragment-read pipelining - goldens + stem tests, stem timing (both trunks), C1 latency
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_ops_gpu.py -v -m gpu -x --timeout 240 --timeout-method thread -k "forward_matches_reference_goldens or stem_pool or nchw_stem" > gpurun_out/r5g_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; grep -E "passed|failed|Error|max err" gpurun_out/r5g_tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for v in "0 0" "1 0" "0 1"; do
  set -- $v
  DDMI_STEM_DIAG=$1 DDMI_STEM1=$2 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r5g_stem_d$1_o$2" -- python3 "$R/tools/micro/stem_time.py" > "$R/gpurun_out/r5g_stem_d$1_o$2.log" 2>&1
  rc=$?; echo "[stem diag=$1 one=$2] rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
cd "$R"
timeout -k 10 300 python -u tools/bench_configs.py --c1-child --c1-streams 2 --steps 20 > gpurun_out/r5g_c1.log 2>&1
rc=$?; echo "[c1] rc=$rc"; grep C1TWO gpurun_out/r5g_c1.log; exit $rc
