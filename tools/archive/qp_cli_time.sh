#!/bin/bash
# End-to-end timing of the quickprobs drop-in on a synthetic family (GPU box):
#   tools/qp_cli_time.sh N LEN [ref]
# With `ref`, the reference QuickProbs CLI built from source
# (oracle/_ref/quickprobs, -t 16) runs on the same input and the two FASTA
# outputs are compared byte for byte.
set -e -o pipefail
N=${1:-128}; L=${2:-256}; REF=${3:-}
mkdir -p gpurun_out
F=gpurun_out/qpfam_${N}_${L}
python3 -c "
import sys; sys.path.insert(0, '.')
from mlprobs_amd import synth
synth.write_fasta('$F.fa', synth.family($N, $L, 0.7, seed=11))
"
t0=$(date +%s.%N)
MLP_CLI_TIMES=1 ./mlprobs_amd/cli/quickprobs $F.fa > $F.gpu.fa 2> $F.err
t1=$(date +%s.%N)
echo "quickprobs (GPU) N=$N L=$L wall $(awk "BEGIN{print $t1 - $t0}") s" | tee $F.time
cat $F.err >> $F.time
if [ -n "$REF" ]; then
  t0=$(date +%s.%N)
  ./oracle/_ref/quickprobs -t 16 $F.fa > $F.ref.fa
  t1=$(date +%s.%N)
  echo "reference quickprobs (CPU, 16 threads) N=$N L=$L wall $(awk "BEGIN{print $t1 - $t0}") s" | tee -a $F.time
  if cmp -s $F.gpu.fa $F.ref.fa; then echo "outputs identical" | tee -a $F.time; else echo "OUTPUTS DIFFER" | tee -a $F.time; fi
fi
