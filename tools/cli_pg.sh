#!/bin/bash
# CLI posterior stage at C3 with the PF posterior in the Zm slots vs its own array
export TMPDIR=/tmp
O=gpurun_out/cli_pg; mkdir -p $O
FA=tests/golden/config/c3_512x400_s11.fa
for rep in 1 2; do for pgs in 0 1; do
  MLP_TEST_PG_SEPARATE=$pgs MLP_CLI_TIMES=1 timeout -k 10 120 mlprobs_amd/cli/c_p_np_aln -p 0 $FA > $O/out_$pgs.msa 2> $O/err_$pgs.txt || exit 1
  echo "pg_separate=$pgs run $rep: $(grep -E '^\[stage\] (posteriors|consistency) ' $O/err_$pgs.txt | tr '\n' ' ') $(cmp -s $O/out_$pgs.msa tests/golden/config/c3_512x400_s11.p_0.out && echo identical)" | tee -a $O/summary.txt
done; done
