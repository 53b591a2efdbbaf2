#!/bin/bash
# round 5k: r5i (decoder groups / union split A/B at B = 64) then r5j (union value_proj timing diagnostics)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
bash tools/gpu_r5j.sh || exit $?
bash tools/gpu_r5i.sh
