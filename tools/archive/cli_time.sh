#!/bin/bash
# End-to-end timing of the c_p_np_aln drop-in on a synthetic family
# (GPU box): tools/cli_time.sh N LEN [extra c_p_np_aln flags]
set -e
N=${1:-512}; L=${2:-400}; shift 2 || true
mkdir -p gpurun_out
F=gpurun_out/fam_${N}_${L}
python3 -c "
import sys; sys.path.insert(0, '.')
from mlprobs_amd import synth
synth.write_fasta('$F.fa', synth.family($N, $L, 0.7, seed=11))
"
t0=$(date +%s.%N)
MLP_CLI_TIMES=1 ./mlprobs_amd/cli/c_p_np_aln -p 0 "$@" $F.fa > $F.mfa 2> $F.err
t1=$(date +%s.%N)
echo "N=$N L=$L wall $(awk "BEGIN{print $t1 - $t0}") s" | tee $F.time
cat $F.err >> $F.time
