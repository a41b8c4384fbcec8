#!/bin/bash
# The quickprobs drop-in on C3: stage split and the host breakdown of
# construction + refinement (MLP_CLI_TIMES), three runs, then one run under
# rocprofv3's kernel trace.   tools/qp_stages.sh -> gpurun_out/qp_stages/
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/qp_stages
mkdir -p $O
FA=tests/golden/config/c3_512x400_s11.fa
CLI=mlprobs_amd/cli/quickprobs
for rep in 1 2 3; do
  MLP_CLI_TIMES=1 timeout -k 10 120 $CLI $FA > $O/out_$rep.fa 2> $O/err_$rep.txt || { tail -5 $O/err_$rep.txt; exit 1; }
  echo "run $rep"; grep -E '^\[(stage|host)\]' $O/err_$rep.txt
done | tee $O/summary.txt
MLP_CLI_TIMES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o qp -- $CLI $FA \
  > $O/trace_out.fa 2> $O/trace_err.txt || { tail -5 $O/trace_err.txt; exit 1; }
