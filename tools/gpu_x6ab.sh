#!/bin/bash
# conv_x6 A/B on one box: per-tile kernel (DDMI_X6_PERSIST=0) vs persistent, alternated twice
set -u
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
for r in 1 2; do
  for p in 0 1; do
    DDMI_X6_PERSIST=$p timeout -k 10 100 tools/micro/conv_bench 10 ${F:-3x3} > gpurun_out/ab.log 2>&1 || { cat gpurun_out/ab.log; exit 1; }
    echo "== persist $p"; grep -v "^shape" gpurun_out/ab.log | awk '{printf "%s %s | ", $1, $2} END {print ""}'
  done
done
