#!/bin/bash
# conv_x5 software-pipelined chunk walk (DDMI_X5_PIPE=1, read per dispatch): the conv / GEMM op tests with it on, the
# conv_x5 shapes of the conv micro-benchmark (off / on / off, same box), then the bench A/B.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 env DDMI_X5_PIPE=1 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q -k "conv or gemm or linear" \
  --timeout 200 --timeout-method thread > gpurun_out/x5pipe_test.log 2>&1; rc=$?
tail -3 gpurun_out/x5pipe_test.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/x5pipe.log; : > $out
for shp in gpt.mlp0 gpt.qkv4 gpt.mlp2 gpt.proj4 gpt.mlp0s3 gpt.qkv3 gpt.qkv2 gpt.mlp0s2 img.l2.s2 img.l3.s2; do
  for v in "DDMI_X5_PIPE=0" "DDMI_X5_PIPE=1" "DDMI_X5_PIPE=0" "DDMI_X5_PIPE=1"; do
    r=$(env $v timeout -k 5 60 tools/micro/conv_bench 20 $shp 2>&1 | grep "^$shp "); rc=$?
    [ $rc -ne 0 ] && { echo "rc=$rc $shp $v"; exit $rc; }
    echo "[$v] $r" | tee -a $out
  done
done
STEPS=100 bash tools/gpu_envab.sh "DDMI_X5_PIPE=0" "DDMI_X5_PIPE=1" | tee gpurun_out/envab_x5pipe.txt
