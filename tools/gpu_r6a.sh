set -o pipefail
mkdir -p gpurun_out/dot
timeout -k 10 120 ./tools/repro/memset_node 500 50 gpurun_out/dot > gpurun_out/r6a_memset.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_parity_gpu.py -k "resnet50_config or reference_goldens" > gpurun_out/r6a_tests.log 2>&1
rc=$?; cat gpurun_out/r6a_memset.log; tail -30 gpurun_out/r6a_tests.log; exit $rc
