#!/bin/bash
# GPU box: SQ counter passes over a short single-stream bench (summarise with tools/pmc_db.py / pmc_dump.py).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p "$R/gpurun_out/pmcb"
cd /tmp && export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
            "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS" \
            "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_WAVES"; do
  i=$((i+1))
  DDMI_STREAMS=0 timeout -s KILL 120 rocprofv3 --pmc $ctrs -f csv -d "$R/gpurun_out/pmcb/p$i" -o run -- python "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-compare > "$R/gpurun_out/pmcb/p$i.log" 2>&1
  rc=$?; echo "[pass $i] rc=$rc"; [ $rc -ne 0 ] && tail -3 "$R/gpurun_out/pmcb/p$i.log" && exit $rc
done
exit 0
