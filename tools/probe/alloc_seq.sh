#!/bin/bash
# Back-to-back fresh processes allocating (hipMalloc) and first-touching
# (hipMemset) device memory: where does a process wait for memory an earlier
# process released, and does the wait scale with the chunk or the total?
#   tools/probe/alloc_seq.sh -> gpurun_out/alloc_seq/summary.txt
set -o pipefail
O=gpurun_out/alloc_seq
mkdir -p $O
P=tools/probe/alloc_chunks
one() {  # chunk_gb total_gb
  local t0=$(date +%s.%N)
  timeout -k 10 60 $P "$@" > $O/last.txt 2>&1 || { cat $O/last.txt; exit 1; }
  local t1=$(date +%s.%N)
  echo "== alloc_chunks $* wall $(awk "BEGIN{print $t1 - $t0}")" >> $O/summary.txt
  awk '{ if ($0 ~ /chunk/) { n++; if (n <= 3 || $6 > 0.2 || $8 > 0.2) print } else print }' $O/last.txt >> $O/summary.txt
}
for k in 1 2 3; do one 32 32; done
for k in 1 2 3; do one 16 16; done
for k in 1 2 3; do one 2 32; done
for k in 1 2 3; do one 32 32; done
for k in 1 2 3; do one 0.5 32; done
for k in 1 2; do one 32 48; done
for k in 1 2; do one 16 48; done
cat $O/summary.txt
