# round 6 (aj): conv_x6 LiDAR layer-3 / layer-4 forms (DDMI_X6_ALT, temporary): 0 = routed (8-wave 32 x 32 / 64 x 32
# wave tiles), 1 = the 8 x 8 maps on 4 waves of 32 x 64, 2 = the 16 x 16 BN = 64 maps on the two-per-CU 4-wave form
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for v in 0 1 2 0 1 2; do
  DDMI_X6_ALT=$v timeout -k 10 120 ./tools/micro/conv_bench 40 lid.l > gpurun_out/r6aj_$v.log 2>&1 || { cat gpurun_out/r6aj_$v.log; exit 1; }
  echo "[alt $v]"; grep -E "3x3|shape" gpurun_out/r6aj_$v.log
done
