set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -v -m gpu -x --timeout 240 --timeout-method thread -k "value_proj_variants or forward_matches_reference_goldens or layernorm_fold or fused_basicblock" > gpurun_out/r5c_vp_tests.log 2>&1
rc=$?; echo "[vp tests] rc=$rc"; tail -3 gpurun_out/r5c_vp_tests.log; grep -A30 "gathered value_proj" gpurun_out/parity_report.txt | head -40; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/r5c_bench.log 2>&1
rc=$?; echo "[bench] rc=$rc"; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_diag_mk.sh r5c
