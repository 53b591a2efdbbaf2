#!/bin/bash
# GPU box: conv_bench on the GPT GEMM shapes and the 8x8 LiDAR conv, default routing vs conv_x5 tile overrides.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
for t in ${TILES:-"" 1 2 3 4}; do
  echo "== DDMI_X5_TILE=$t"
  DDMI_X5_TILE=$t timeout -k 10 120 "$R/tools/micro/conv_bench" 10 ${F:-gpt} || exit $?
  DDMI_X5_TILE=$t timeout -k 10 120 "$R/tools/micro/conv_bench" 10 lid.l4 || exit $?
done
