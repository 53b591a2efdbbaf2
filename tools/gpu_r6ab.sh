# round 6 (ab): the small-N GPT GEMMs (C = 64 / 128 / 256 blocks) on conv_x5 64 x 64 / 64 x 128 tiles with 3-4 LDS-DMA
# stages at two-three workgroups per CU (DDMI_X5_SMALLN = 3 / 4 / 5) against their routes (conv_x3 / conv_x5)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for w in 0 3 4 5; do
  DDMI_X5_SMALLN=$w timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/r6ab_$w" -- python3 "$R/tools/micro/gemm_shapes.py" > "$R/gpurun_out/r6ab_$w.log" 2>&1 || { tail -5 "$R/gpurun_out/r6ab_$w.log"; exit 1; }
  echo "[SMALLN=$w]"; grep -c "rel err" "$R/gpurun_out/r6ab_$w.log"; python3 "$R/tools/micro/gemm_shapes.py" --parse "$R/gpurun_out/r6ab_$w"; rm -rf "$R/gpurun_out/r6ab_$w"
done
