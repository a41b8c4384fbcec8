#!/bin/bash
# r05 GPU call: c_p_np_aln device-MEA floor after the pinned-buffer fix -- C2 -p 0 / -p 1, floors 2.5e5 / 5e4 / 0,
# stage times, outputs against the reference's
set -o pipefail
export TMPDIR=/tmp MLP_SRAND_TIME=1700000000
O=gpurun_out/floor; mkdir -p $O
c=c2_128x256_s11; FA=tests/golden/config/$c.fa
for k in 1 2 3; do for mode in 0 1; do for m in 250000 50000 0; do
  MLP_MEA_GPU_MIN=$m MLP_CLI_TIMES=1 timeout -k 10 120 mlprobs_amd/cli/c_p_np_aln -p $mode $FA > $O/o.msa 2> $O/e.txt || { tail -5 $O/e.txt; exit 1; }
  echo "-p $mode floor $m run $k: $(grep -E '^\[stage\] (progressive \+ refinement|refinement|context teardown)' $O/e.txt | tr '\n' ' ') $(grep '^\[host\]' $O/e.txt) $(cmp -s $O/o.msa tests/golden/config/$c.p_$mode.out && echo identical-to-ref)" | tee -a $O/summary.txt
done; done; done
