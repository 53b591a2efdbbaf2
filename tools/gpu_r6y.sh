# round 6 (y): the 1x1 stride-2 downsamples on conv_x5's 128 x 128 two-per-CU tiles (DDMI_X5_DS128=1) vs their routes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for w in 0 1 0 1; do
  DDMI_X5_DS128=$w timeout -k 10 120 ./tools/micro/conv_bench 20 .ds > gpurun_out/r6y_$w.log 2>&1 || { cat gpurun_out/r6y_$w.log; exit 1; }
  echo "[DS128=$w]"; grep -v amdgpu.ids gpurun_out/r6y_$w.log
done
