#!/bin/bash
# GPU box: PMC counters of the x6 conv kernel on one shape (separate passes, each under its own timeout).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p "$R/gpurun_out/pmc6"
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" \
            "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs -d "$R/gpurun_out/pmc6/p$i" -o run -- "$R/tools/micro/conv_bench" 3 ${F:-img.l3} > "$R/gpurun_out/pmc6/p$i.log" 2>&1
  rc=$?; echo "[pass $i] rc=$rc"; tail -2 "$R/gpurun_out/pmc6/p$i.log"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
