# round 6 (p): the stem's XCD-aware tile walk - bit-identity against the previous build, kernel times, then PMC passes
# (MFMA busy, LDS conflicts, HBM read / write bytes, L2 hit) of both builds' stems (tools/micro/stem_ab.py, REPS=3)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
OLD=$R/tools/micro/ab/old/libddmi.so
DDMI_LIB=$OLD OUT=gpurun_out/r6p_old.json timeout -k 10 200 python tools/micro/stem_ab.py > gpurun_out/r6p_ab.log 2>&1 || { cat gpurun_out/r6p_ab.log; exit 1; }
OUT=gpurun_out/r6p_new.json REF=gpurun_out/r6p_old.json timeout -k 10 200 python tools/micro/stem_ab.py >> gpurun_out/r6p_ab.log 2>&1 || { cat gpurun_out/r6p_ab.log; exit 1; }
grep bit-identical gpurun_out/r6p_ab.log
cd /tmp && export TMPDIR=/tmp
for v in old new; do
  if [ $v = old ]; then export DDMI_LIB=$OLD; else unset DDMI_LIB; fi
  OUT=/tmp/x.json timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r6p_$v" -- python3 "$R/tools/micro/stem_ab.py" > "$R/gpurun_out/r6p_$v.log" 2>&1 || exit 1
  echo "[$v]"; python3 "$R/tools/kstats.py" "$R/gpurun_out/r6p_$v" --grep stem_pool
  i=0
  for ctrs in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    REPS=3 OUT=/tmp/x.json timeout -s KILL 120 rocprofv3 --pmc $ctrs --kernel-trace -f csv -d "$R/gpurun_out/r6p_pmc_$v/p$i" -o run -- python3 "$R/tools/micro/stem_ab.py" > "$R/gpurun_out/r6p_pmc_$v/p$i.log" 2>&1 || { echo "pmc pass $i rc=$?"; exit 1; }
  done
  python3 "$R/tools/pmc_kernels.py" "$R/gpurun_out/r6p_pmc_$v" --grep stem_pool
done
