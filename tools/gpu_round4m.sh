#!/bin/bash
# Round-4 (m): host AddressSanitizer over the library's host code (tools/repro/asan_driver: every gemm mode, B 1/4/8,
# heads, single-stream lanes on a caller stream, the training forward, a long-lived handle), then - if clean - the
# whole GPU suite in its default order with the dbg library, uncaptured, to place the full-suite fault (pool on).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
python - <<'PY' || exit 1
from diffusiondrive_amd.config import TransfuserConfig
from diffusiondrive_amd.weights import seeded_state_dict, pack_blob
open("/tmp/dd_w.ddw1", "wb").write(pack_blob(seeded_state_dict(TransfuserConfig(), 0)))
PY
timeout -k 10 900 env ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0:halt_on_error=1 tools/repro/asan_driver \
  /tmp/dd_w.ddw1 45 > gpurun_out/asan.log 2>&1
rc=$?; echo "[asan] rc=$rc"; tail -3 gpurun_out/asan.log; grep -m3 -n "ERROR: AddressSanitizer" gpurun_out/asan.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 env DDMI_LIB=$R/diffusiondrive_amd/_variants/libddmi_dbg.so python -u -m pytest tests -v -s -m gpu -x \
  --timeout 300 --timeout-method thread > gpurun_out/suite_dbg.log 2>&1
rc=$?; echo "[suite_dbg] rc=$rc"; grep -n -A12 "SIGSEGV backtrace" gpurun_out/suite_dbg.log | head -20; tail -2 gpurun_out/suite_dbg.log
exit $rc
