# round 6 (n): the GPT-shaped GEMMs (conv_x5 / conv_x3) against hipBLASLt's fp16 GEMM at K' = 3K, kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r6n_gemm" -- python3 "$R/tools/micro/gemm_vs_blaslt.py" > "$R/gpurun_out/r6n_gemm.log" 2>&1
rc=$?; echo "[gemm] rc=$rc"; grep -v amdgpu.ids "$R/gpurun_out/r6n_gemm.log"; python3 "$R/tools/kstats.py" "$R/gpurun_out/r6n_gemm" | head -40; exit $rc
