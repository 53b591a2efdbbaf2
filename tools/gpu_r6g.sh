# round 6 (g): the memset-node reproducer with the memset in the middle of the graph (cases 9 / 10)
set -o pipefail
for w in 16 64; do
  timeout -k 10 120 ./tools/repro/memset_node 500 20 - $w > gpurun_out/r6g_memset_w$w.log 2>&1 || exit $?
  echo "words $w:"; grep "case [0-9]*:" gpurun_out/r6g_memset_w$w.log | grep -v "case [0-6]:"
done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 120 ./tools/repro/memset_node 500 20 - 16 > gpurun_out/r6g_memset_nopc.log 2>&1
echo "packet capture off:"; grep "case \(9\|10\)" gpurun_out/r6g_memset_nopc.log
