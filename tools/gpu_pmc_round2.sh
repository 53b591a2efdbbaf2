#!/bin/bash
# GPU box: per-kernel PMC counters of the bench workload (B = 64, single-stream replays), one rocprofv3 pass
# per counter group with the kernel trace only beside --pmc (MI355X_MICROARCH.md "rocprofv3 PMC slots":
# <= 8 SQ, <= 4 TCC with FETCH_SIZE = 3 and WRITE_SIZE = 2, <= 2 GRBM per pass). Summarise afterwards with
#   python tools/pmc_round2.py gpurun_out/pmc2 round2_pmc
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p "$R/gpurun_out/pmc2"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-compare --in-flight 1"
i=0
for ctrs in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_GUI_ACTIVE GRBM_COUNT" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
            "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  DDMI_STREAMS=0 timeout -s KILL 240 rocprofv3 --pmc $ctrs --kernel-trace -f csv -d "$R/gpurun_out/pmc2/p$i" -o run -- python "$R/bench.py" $ARGS > "$R/gpurun_out/pmc2/p$i.log" 2>&1
  rc=$?; echo "[pass $i: $ctrs] rc=$rc"; tail -1 "$R/gpurun_out/pmc2/p$i.log" | cut -c1-200
  [ $rc -ne 0 ] && exit $rc
done
exit 0
