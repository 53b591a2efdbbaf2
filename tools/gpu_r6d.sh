# round 6 (d): the memset-node reproducer with the tfdec_mk4 counter pattern (cases 7 / 8), graph packet capture on
# (the runtime default) and off
set -o pipefail
timeout -k 10 120 ./tools/repro/memset_node 500 20 > gpurun_out/r6d_memset.log 2>&1 && \
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 120 ./tools/repro/memset_node 500 20 > gpurun_out/r6d_memset_nopc.log 2>&1
rc=$?; cat gpurun_out/r6d_memset.log; echo "--- packet capture off"; cat gpurun_out/r6d_memset_nopc.log; exit $rc
