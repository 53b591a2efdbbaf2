#!/bin/bash
# GPU box: secondary configs C1 / C2 / C4 / C5 / C6 (tools/bench_configs.py) -> gpurun_out/configs.{json,md}
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 900 python tools/bench_configs.py > gpurun_out/configs.log 2>&1
rc=$?; echo "[configs] rc=$rc"; tail -5 gpurun_out/configs.log; exit $rc
