#!/bin/bash
# Round-3 (p) evidence: tools/gpu_all.sh (GPU tests, bench, rocprof trace), then the PMC passes. Stops at the first
# abnormal exit.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
bash tools/gpu_all.sh || exit $?
cd "$R" && bash tools/gpu_pmc_round2.sh
