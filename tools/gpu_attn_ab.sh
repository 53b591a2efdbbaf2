#!/bin/bash
# GPT attention micro-benchmark A/B (tools/micro/attn_bench.py): score operand splits and waves per workgroup
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for cfg in "$@"; do
  echo "[$cfg]"
  env $cfg timeout -k 10 120 python tools/micro/attn_bench.py || exit $?
done
