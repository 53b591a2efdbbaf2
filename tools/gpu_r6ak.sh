# round 6 (ak): conv_x6 small-grid form (DDMI_X6_SMALL=2: 8 x 8 pixel tiles x 64 channels, 4 waves) against the routed
# forms on the LiDAR trunk's 3x3 shapes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for v in 1 2 1 2; do
  DDMI_X6_SMALL=$v timeout -k 10 120 ./tools/micro/conv_bench 40 3x3 > gpurun_out/r6ak_$v.log 2>&1 || { cat gpurun_out/r6ak_$v.log; exit 1; }
  echo "[small $v]"; grep -E "3x3|shape" gpurun_out/r6ak_$v.log
done
