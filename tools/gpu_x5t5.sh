#!/bin/bash
# conv micro-benchmark: the GPT N=512 GEMMs (scale 4 proj / MLP-down) and the other M=20480 shapes on the current
# routing vs the 192 x 256 tile (DDMI_X5_TILE=5)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for shp in ${SHAPES:-gpt.mlp2 gpt.proj4 gpt.mlp0 gpt.qkv4 gpt.mlp0s3 gpt.mlp2s3 gpt.qkv3 gpt.mlp0s2 gpt.qkv2 gpt.proj3}; do
  for t in ${TILES:-0 5 6}; do
    out=$(DDMI_X5_TILE=$t timeout -k 5 60 tools/micro/conv_bench ${REPS:-30} $shp 2>&1)
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc $shp $t"; echo "$out"; exit $rc; }
    echo "$out" | awk -v s="$shp" -v t="$t" '$1 == s { print "tile=" t " " $0 }'
  done
done
