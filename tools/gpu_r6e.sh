# round 6 (e): counter tests (kernel-node-only program, dirty counters flagged and healed, forced timeouts), the
# in-flight lanes and the query-group tests on the sc1 hand-off
set -o pipefail
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_sync_gpu.py tests/test_inflight_gpu.py tests/test_parity_gpu.py -k "sync or kernel_nodes or inflight or groups or graph_replay" > gpurun_out/r6e_tests.log 2>&1
rc=$?; tail -40 gpurun_out/r6e_tests.log; exit $rc
