#!/bin/bash
# stem_pool LDS-conflict share per library build (rocprofv3 --pmc on tools/micro/stem_op.py): product, then variants
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p "$R/gpurun_out/stpmc"
cd /tmp && export TMPDIR=/tmp
for v in "" "$@"; do
  L=$R/diffusiondrive_amd/libddmi${v:+_$v}.so
  DDMI_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS --kernel-trace -f csv -d "$R/gpurun_out/stpmc/${v:-base}" -o run -- python "$R/tools/micro/stem_op.py" > "$R/gpurun_out/stpmc/${v:-base}.log" 2>&1
  rc=$?; echo "[${v:-base}] rc=$rc $(tail -1 $R/gpurun_out/stpmc/${v:-base}.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
