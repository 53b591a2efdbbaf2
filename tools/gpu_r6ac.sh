# round 6 (ac): the GPT attention with two LDS stages at every head size (DDMI_ATTN_NB2=1) vs one stage for hs >= 64
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for w in 0 1 0 1; do
  DDMI_ATTN_NB2=$w timeout -k 10 120 python tools/micro/attn_bench.py > gpurun_out/r6ac_$w.log 2>&1 || { cat gpurun_out/r6ac_$w.log; exit 1; }
  echo "[NB2=$w]"; grep -v amdgpu.ids gpurun_out/r6ac_$w.log
done
