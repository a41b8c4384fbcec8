#!/bin/bash
# Where a fresh c_p_np_aln / quickprobs process spends its time on small
# families (GPU box): wall clock around the process and the stage times
# (MLP_CLI_TIMES), against the reference CLI's wall clock.
#   tools/e2e_small.sh -> gpurun_out/e2e_small/summary.txt
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/e2e_small
mkdir -p $O
CLI=./mlprobs_amd/cli/c_p_np_aln
REF=./oracle/_ref/c_p_np_aln
for fa in tests/golden/edge/two.fa tests/golden/real/ox_104s10.fa tests/golden/real/sabre_sup_017.fa \
          tests/golden/cli/bb11028.fa tests/golden/config/c2_128x256_s11.fa; do
  for run in 1 2; do
    t0=$(date +%s.%N)
    timeout -k 10 120 env MLP_CLI_TIMES=1 $CLI -p 0 $fa > /dev/null 2> $O/err.txt || { cat $O/err.txt; exit 1; }
    t1=$(date +%s.%N)
    echo "$fa drop-in run $run wall $(awk "BEGIN{print $t1 - $t0}")" >> $O/summary.txt
    grep '^\[stage\]' $O/err.txt >> $O/summary.txt
  done
  t0=$(date +%s.%N)
  timeout -k 10 300 $REF -p 0 $fa > /dev/null 2>&1
  t1=$(date +%s.%N)
  echo "$fa reference wall $(awk "BEGIN{print $t1 - $t0}")" >> $O/summary.txt
done
# the runtime alone: a process that only initialises HIP
t0=$(date +%s.%N)
timeout -k 10 60 python3 -c "import ctypes; l=ctypes.CDLL('./mlprobs_amd/lib/libmlpgpu.so'); print(l)" > /dev/null
t1=$(date +%s.%N)
echo "dlopen libmlpgpu (python) wall $(awk "BEGIN{print $t1 - $t0}")" >> $O/summary.txt
cat $O/summary.txt
