# round 6 (a): memset-node ordering reproducer, tf_replay with the memset node back (does the new counter check flag
# the failing replays?), the C4 goldens and the query-group / tf-decoder-group tests
set -o pipefail
mkdir -p gpurun_out/dot
timeout -k 10 120 ./tools/repro/memset_node 500 50 gpurun_out/dot > gpurun_out/r6a_memset.log 2>&1 && \
DDMI_TF_MEMSET=1 timeout -k 10 300 python -u tools/debug/tf_replay.py > gpurun_out/r6a_tfr_memset.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_parity_gpu.py -k "resnet50_config or reference_goldens or groups" > gpurun_out/r6a_tests.log 2>&1
rc=$?; cat gpurun_out/r6a_memset.log; grep -c "same-as-first False" gpurun_out/r6a_tfr_memset.log; grep "streams 2" gpurun_out/r6a_tfr_memset.log | head -12; tail -30 gpurun_out/r6a_tests.log; exit $rc
