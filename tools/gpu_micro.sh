#!/bin/bash
# GPU box: conv microbenchmark, default dispatch vs variants. Stops at the first abnormal exit.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for v in "${@:-default}"; do
  case $v in
    default) envs="";;
    *) envs="$v";;
  esac
  echo "== $v"
  env $envs timeout -k 10 120 tools/micro/conv_bench 20 > "gpurun_out/micro_$v.log" 2>&1
  rc=$?; cat "gpurun_out/micro_$v.log"
  if [ $rc -ne 0 ]; then echo "rc=$rc: stopping"; exit $rc; fi
done
