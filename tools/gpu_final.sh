#!/bin/bash
# Round-end evidence on one box: every GPU test, the bench line, the rocprofv3 kernel trace of the bench workload
# (tools/gpu_all.sh), then the PMC passes (tools/gpu_pmc_round2.sh). Stops at the first abnormal exit.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
bash tools/gpu_all.sh || exit $?
cd "$R" && bash tools/gpu_pmc_round2.sh
