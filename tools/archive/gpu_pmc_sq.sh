#!/bin/bash
# SQ / TCC counters per kernel for one profiled forward (tools/launch_log.py), one rocprofv3 pass per
# counter group (kernel trace only beside --pmc). Args: extra launch_log args (e.g. --gemm f16x3).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
i=0
PGROUPS=${PMC_GROUPS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES;SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM;SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM;TCC_HIT_sum TCC_MISS_sum"}
IFS=';' read -ra GRPS <<< "$PGROUPS"
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -f csv -d "$R/gpurun_out/sq$i" -o run -- python "$R/tools/launch_log.py" --reps 1 --out "$R/gpurun_out/ll_sq$i.md" "$@" > "$R/gpurun_out/sq$i.log" 2>&1
  rc=$?; echo "[pass $i: $grp] rc=$rc"; tail -2 "$R/gpurun_out/sq$i.log"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
