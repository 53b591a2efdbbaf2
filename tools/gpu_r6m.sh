# round 6 (m): after reverting the conv_x6 DMA-halo / persistent experiment - the shipped conv_x6 forms on the
# micro-benchmark (time + error vs fp32), then the whole-tree check
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 120 ./tools/micro/conv_bench 20 3x3 > gpurun_out/r6m_conv.log 2>&1
rc=$?; echo "[conv_bench] rc=$rc"; grep -v amdgpu.ids gpurun_out/r6m_conv.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_check.sh r6m
