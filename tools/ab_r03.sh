#!/bin/bash
# Round-3 A/B pass on the GPU box:
#   1. posterior stage with the side stream joined after each sweep (MLP_JOIN=0),
#      joined before the merge (1) and as per-model chains (2), alternating;
#   2. quickprobs C3 end to end with the host MEA and the device MEA
#      (MLP_MEA_DEVICE=1), alternating, outputs compared;
#   3. the allocation probe sequence (tools/probe/alloc_seq.sh).
#   tools/ab_r03.sh [parts...] -> gpurun_out/ab/summary.txt
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
PARTS=${*:-"join mea alloc"}
F3=tests/golden/config/c3_512x400_s11.fa
for part in $PARTS; do
case $part in
join)
  for rep in 1 2; do
    for j in 0 1 2; do
      MLP_JOIN=$j timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --no-qp --relax 0 --no-shards --steps 3 --warmup 1 \
        > $O/join$j.json 2> $O/join$j.err || { tail -5 $O/join$j.err; exit 1; }
      python3 -c "
import json; d=json.load(open('$O/join$j.json'))
k=d['kernels_ms_per_step']
print('MLP_JOIN=$j', 'step %.1f ms' % d['ms_per_step'], ' '.join('%s %.1f' % (a, b) for a, b in k.items()), 'parity', d.get('parity', {}).get('bit_exact_pairs', ''))" | tee -a $O/summary.txt
    done
  done ;;
mea)
  for rep in 1 2; do
    for m in 0 1; do
      t0=$(date +%s.%N)
      MLP_MEA_DEVICE=$m MLP_CLI_TIMES=1 timeout -k 10 120 ./mlprobs_amd/cli/quickprobs $F3 > $O/qp$m.out 2> $O/qp$m.err || { tail -5 $O/qp$m.err; exit 1; }
      t1=$(date +%s.%N)
      echo "quickprobs C3 MLP_MEA_DEVICE=$m wall $(awk "BEGIN{print $t1 - $t0}")" | tee -a $O/summary.txt
      grep -E 'construction|\[host\]|posteriors' $O/qp$m.err | tee -a $O/summary.txt
    done
    cmp $O/qp0.out $O/qp1.out && echo "quickprobs C3 host / device MEA outputs identical" | tee -a $O/summary.txt
  done ;;
jointest)
  for j in 1 2; do
    MLP_JOIN=$j timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
      > $O/jointest$j.log 2>&1 || { tail -20 $O/jointest$j.log; exit 1; }
    echo "MLP_JOIN=$j parity tests: $(tail -1 $O/jointest$j.log)" | tee -a $O/summary.txt
  done ;;
alloc)
  tools/probe/alloc_seq.sh > /dev/null && cat gpurun_out/alloc_seq/summary.txt >> $O/summary.txt ;;
esac
done
cat $O/summary.txt
