#!/bin/bash
# r05 GPU call: host sparse set with uninitialised row pointers (filled by mlp_csr_export) against the previous
# binary (c_p_np_aln_old): C3 -p 0 / -p 1 "sparse set to host" stage, outputs against the reference
set -o pipefail
export TMPDIR=/tmp MLP_SRAND_TIME=1700000000
O=gpurun_out/noinit; mkdir -p $O
FA=tests/golden/config/c3_512x400_s11.fa
for k in 1 2 3; do for v in old new; do
  B=mlprobs_amd/cli/c_p_np_aln; [ $v = old ] && B=mlprobs_amd/cli/c_p_np_aln_old
  MLP_CLI_TIMES=1 timeout -k 10 120 $B -p 0 $FA > $O/o.msa 2> $O/e.txt || { tail -5 $O/e.txt; exit 1; }
  echo "$v run $k: $(grep -E '^\[stage\] (sparse set to host|posteriors) ' $O/e.txt | tr '\n' ' ') $(cmp -s $O/o.msa tests/golden/config/c3_512x400_s11.p_0.out && echo identical)" | tee -a $O/summary.txt
done; done
C2=tests/golden/config/c2_128x256_s11.fa
mlprobs_amd/cli/c_p_np_aln -p 1 $C2 > $O/c2.msa && cmp $O/c2.msa tests/golden/config/c2_128x256_s11.p_1.out && echo "C2 -p 1 identical"
