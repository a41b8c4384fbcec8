#!/bin/bash
# The c_p_np_aln drop-in's posterior stage on C3 against its batch scratch
# (MLP_SCRATCH_GB), then one run at the default 16 GB under rocprofv3's
# kernel trace (per-batch kernel durations and the gaps between them).
#   tools/cli_batches.sh [GB ...] -> gpurun_out/cli_batches/{summary.txt,trace/}
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/cli_batches
mkdir -p $O
FA=tests/golden/config/c3_512x400_s11.fa
CLI=mlprobs_amd/cli/c_p_np_aln
for gb in "${@:-16 24 32 64}"; do
  for rep in 1 2; do
    MLP_CLI_TIMES=1 MLP_SCRATCH_GB=$gb timeout -k 10 120 $CLI -p 0 $FA > $O/out_$gb.msa 2> $O/err_$gb.txt || { tail -5 $O/err_$gb.txt; exit 1; }
    echo "scratch ${gb} GB run $rep: $(grep -E '^\[stage\] (posteriors|consistency) ' $O/err_$gb.txt | tr '\n' ' ')" | tee -a $O/summary.txt
  done
  cmp -s $O/out_$gb.msa tests/golden/config/c3_512x400_s11.p_0.out && echo "  output identical to the reference CLI's" | tee -a $O/summary.txt
done
MLP_CLI_TIMES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o cli -- $CLI -p 0 $FA \
  > $O/trace_out.msa 2> $O/trace_err.txt || { tail -5 $O/trace_err.txt; exit 1; }
grep -E '^\[stage\] ' $O/trace_err.txt | tee -a $O/summary.txt
