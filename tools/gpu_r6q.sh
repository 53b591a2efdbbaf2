# round 6 (q): conv_x5 256 x 256 as 4 waves of 128 x 128 (DDMI_X5_W4=1) against 8 waves of 64 x 128, GPT shapes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for w in 0 1; do
  DDMI_X5_W4=$w timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/r6q_w$w" -- python3 "$R/tools/micro/gemm_shapes.py" > "$R/gpurun_out/r6q_w$w.log" 2>&1 || { tail -5 "$R/gpurun_out/r6q_w$w.log"; exit 1; }
  echo "[W4=$w]"; grep "rel err" "$R/gpurun_out/r6q_w$w.log" | tr '\n' ' '; echo; python3 "$R/tools/micro/gemm_shapes.py" --parse "$R/gpurun_out/r6q_w$w"; rm -rf "$R/gpurun_out/r6q_w$w"
done
