#!/bin/bash
# One GPU-box session: every -m gpu test, the bench (default args), a single-stream rocprofv3 kernel
# trace of the bench workload, then separate FETCH / WRITE PMC passes. Stops at the first abnormal exit.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash "$R/tools/gpu_all.sh" || exit $?
bash "$R/tools/gpu_pmc.sh"
