#!/bin/bash
# Same-box A/B of library builds through the whole bench (device time per kernel class, wall):
#   gpu_lib_ab.sh <variant> ...   (libddmi_<variant>.so, DDMI_BUILD_VARIANT builds); the product library runs first
#   and last; each variant first runs the gathered-row / golden parity tests ($TESTK).
set -u
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
for v in "$@"; do
  DDMI_LIB=$PWD/diffusiondrive_amd/_variants/libddmi_$v.so timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu \
    -k "${TESTK:-gathered or golden}" --timeout 200 --timeout-method thread > gpurun_out/lab_$v.log 2>&1
  rc=$?; echo "[$v tests] rc=$rc $(tail -1 gpurun_out/lab_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
for l in libddmi.so $(for v in "$@"; do echo _variants/libddmi_$v.so; done) libddmi.so; do
  DDMI_LIB=$PWD/diffusiondrive_amd/$l timeout -k 10 200 python bench.py --steps ${ABSTEPS:-60} --no-cpu-baseline --no-compare ${BENCH_ARGS:-} > gpurun_out/lab.log 2>&1 || { tail -5 gpurun_out/lab.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/lab.log').read().strip().splitlines()[-1]);dm=d['device_ms_per_step'];print('$l', d['value'], d['ms_per_step'], {k: dm[k] for k in ('conv_x6','conv_x5','conv_x3','attn','stem_pool','bilinear')})"
done
