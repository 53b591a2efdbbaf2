#!/bin/bash
# GPU box: conv_bench timings of the 3x3 shapes, then SQ wait / issue counters of one shape (F, default
# img.l3) in separate passes, each under its own timeout.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p "$R/gpurun_out/pmc6"
timeout -k 10 120 "$R/tools/micro/conv_bench" 20 3x3 > "$R/gpurun_out/pmc6/times.log" 2>&1 || exit $?
cat "$R/gpurun_out/pmc6/times.log"
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
            "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS" \
            "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs -d "$R/gpurun_out/pmc6/p$i" -o run -- "$R/tools/micro/conv_bench" 3 ${F:-img.l3} > "$R/gpurun_out/pmc6/p$i.log" 2>&1
  rc=$?; echo "[pass $i] rc=$rc"; tail -1 "$R/gpurun_out/pmc6/p$i.log"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
