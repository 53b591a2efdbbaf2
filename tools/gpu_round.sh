#!/bin/bash
# One GPU-box session: gpu tests, bench, rocprof kernel trace, then separate FETCH/WRITE PMC passes.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash "$R/tools/gpu_all.sh" || exit $?
bash "$R/tools/gpu_pmc.sh"
