set -e -o pipefail
O=gpurun_out/r01t; mkdir -p $O
for i in 1 2 3; do timeout -k 10 120 tools/probe/alloc_probe 140 >> $O/alloc.log 2>&1; done
sleep 15
timeout -k 10 120 tools/probe/alloc_probe 140 >> $O/alloc.log 2>&1
timeout -k 10 120 tools/probe/alloc_probe 24 >> $O/alloc.log 2>&1
timeout -k 10 120 tools/probe/alloc_probe 24 >> $O/alloc.log 2>&1
timeout -k 10 120 tools/probe/alloc_probe 140 >> $O/alloc.log 2>&1
