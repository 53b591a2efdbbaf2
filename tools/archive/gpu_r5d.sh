set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -v -m gpu -x --timeout 240 --timeout-method thread -k "value_proj_variants or forward_matches_reference_goldens or decoder_query_groups or graph_replay" > gpurun_out/r5d_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -3 gpurun_out/r5d_tests.log; grep -A40 "gathered value_proj" gpurun_out/parity_report.txt | grep -E "union|nhalf|trajectory" | head -30; [ $rc -ne 0 ] && exit $rc
for ns in 2; do
  timeout -k 10 300 python -u tools/bench_configs.py --c1-child --c1-streams $ns --steps 20 > gpurun_out/r5d_c1_s$ns.log 2>&1
  rc=$?; echo "[c1 streams=$ns] rc=$rc"; grep C1TWO gpurun_out/r5d_c1_s$ns.log; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/r5d_bench.log 2>&1
rc=$?; echo "[bench] rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/r5d_b1trace" -- python3 "$R/tools/micro/b1_trace.py" > "$R/gpurun_out/r5d_b1trace.log" 2>&1
rc=$?; echo "[b1 trace] rc=$rc"; grep b1_trace "$R/gpurun_out/r5d_b1trace.log"; exit $rc
