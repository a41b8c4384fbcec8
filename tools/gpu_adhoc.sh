#!/bin/bash
# -p 1 at C2 / C3 (GPU posteriors + host alignment graph), stage times
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/p1probe
mkdir -p $O
for f in c2_128x256_s11 c3_512x400_s11; do
  t0=$(date +%s.%N)
  timeout -k 10 400 env MLP_CLI_TIMES=1 ./mlprobs_amd/cli/c_p_np_aln -p 1 tests/golden/config/$f.fa > $O/$f.p1.out 2> $O/$f.p1.err
  rc=$?
  t1=$(date +%s.%N)
  echo "$f -p 1 rc=$rc wall $(awk "BEGIN{print $t1 - $t0}")" | tee -a $O/summary.txt
  grep '^\[stage\]' $O/$f.p1.err | tee -a $O/summary.txt
  [ $rc -eq 0 ] || exit 1
done
