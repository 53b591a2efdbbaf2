# round 6 (q): conv_x5 GEMM tile A/B on the GPT shapes (DDMI_X5_T128=1: 128 x 128 at two workgroups per CU)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for w in 0 1; do
  DDMI_X5_T128=$w timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/r6q_w$w" -- python3 "$R/tools/micro/gemm_shapes.py" > "$R/gpurun_out/r6q_w$w.log" 2>&1 || { tail -5 "$R/gpurun_out/r6q_w$w.log"; exit 1; }
  echo "[T128=$w]"; grep "rel err" "$R/gpurun_out/r6q_w$w.log" | tr '\n' ' '; echo; python3 "$R/tools/micro/gemm_shapes.py" --parse "$R/gpurun_out/r6q_w$w"; rm -rf "$R/gpurun_out/r6q_w$w"
done
