#!/bin/bash
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_parity_gpu.py -v -m gpu -x -rf -k "bf16 or b64_routes or stem or f16x3" --timeout 300 --timeout-method thread > gpurun_out/t_bf16.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -15 gpurun_out/t_bf16.log; grep "==" gpurun_out/parity_report.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --gemm bf16 --no-cpu-baseline --no-compare --steps 10 > gpurun_out/b_bf16_r34.json 2> gpurun_out/b_bf16_r34.err; rc=$?; echo "[bench r34 bf16] rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --arch resnet50 --gemm bf16 --no-cpu-baseline --no-compare --steps 10 > gpurun_out/b_bf16_r50.json 2> gpurun_out/b_bf16_r50.err; rc=$?; echo "[bench r50 bf16] rc=$rc"
python -c "
import json
for f in ['r34','r50']:
    j=json.loads(open('gpurun_out/b_bf16_%s.json'%f).read().strip().splitlines()[-1]); print(f, j['value'], j['ms_per_step'], j['roofline']['kernel'][:8], j['roofline']['achieved'], j['device_ms_per_step'])
"
exit $rc
