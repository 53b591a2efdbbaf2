# round 6 (aa): the C4 (ResNet-50, bf16) forward's conv / GEMM launches with conv_x5's 128 x 128 two-per-CU tiles for
# its bf16 GEMMs and stride-2 convs (DDMI_X5_T128B=1) against the routed tiles
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for w in 0 1; do
  DDMI_X5_T128B=$w timeout -k 10 300 python tools/launch_log.py --arch resnet50 --gemm bf16 --out gpurun_out/r6aa_$w.md > gpurun_out/r6aa_$w.log 2>&1 || { tail -5 gpurun_out/r6aa_$w.log; exit 1; }
  echo "[T128B=$w]"; head -1 gpurun_out/r6aa_$w.md; grep "all shapes\|GEMM / conv total" gpurun_out/r6aa_$w.md
done
