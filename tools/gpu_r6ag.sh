# round 6 (ag): union value_proj, previous build vs residue-class slots: kernel trace of the model A/B forward
# (union kernel and gathered-fallback times) and one PMC pass (MFMA busy, LDS conflicts) per build
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p "$R/gpurun_out/r6ag"
cd /tmp && export TMPDIR=/tmp
for v in old new; do
  if [ $v = old ]; then L="$R/tools/micro/ab/old/libddmi.so"; else L="$R/diffusiondrive_amd/libddmi.so"; fi
  DDMI_LIB=$L OUT=/tmp/ab_$v.json timeout -s KILL 240 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/r6ag/t_$v" -o run -- python "$R/tools/micro/model_ab.py" > "$R/gpurun_out/r6ag/t_$v.log" 2>&1
  rc=$?; echo "[trace $v] rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$R/gpurun_out/r6ag/t_$v.log"; exit $rc; }
  python "$R/tools/kstats.py" "$R/gpurun_out/r6ag/t_$v" --grep vproj
  DDMI_LIB=$L OUT=/tmp/ab_$v.json timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS --kernel-trace -f csv -d "$R/gpurun_out/r6ag/p_$v" -o run -- python "$R/tools/micro/model_ab.py" > "$R/gpurun_out/r6ag/p_$v.log" 2>&1
  rc=$?; echo "[pmc $v] rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$R/gpurun_out/r6ag/p_$v.log"; exit $rc; }
  python "$R/tools/pmc_round2.py" "$R/gpurun_out/r6ag/p_$v" scratch_r6ag_$v | grep -E "value_proj|kernel \|"
done
exit 0
