# round 6 (v): conv_x5 128 x 128 at two workgroups per CU (DDMI_X5_T128=1) on the GPT GEMM shapes and the stride-2
# convs (conv_bench s2), against the routed tiles
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for w in 0 1; do
  DDMI_X5_T128=$w timeout -k 10 120 ./tools/micro/conv_bench 20 s2 > gpurun_out/r6v_s2_$w.log 2>&1 || { cat gpurun_out/r6v_s2_$w.log; exit 1; }
  echo "[T128=$w]"; grep -v amdgpu.ids gpurun_out/r6v_s2_$w.log
done
bash tools/gpu_r6q.sh
