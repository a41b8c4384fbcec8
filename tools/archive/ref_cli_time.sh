#!/bin/bash
# Time the reference C_P_NP_Aln build (oracle/_ref, compiled from the
# reference sources) end to end on a synthetic family, on the GPU box's host
# cores (OMP_NUM_THREADS as set there): tools/ref_cli_time.sh N LEN
set -e
N=${1:-128}; L=${2:-256}
mkdir -p gpurun_out
F=gpurun_out/reffam_${N}_${L}
python3 -c "
import sys; sys.path.insert(0, '.')
from mlprobs_amd import synth
synth.write_fasta('$F.fa', synth.family($N, $L, 0.7, seed=11))
"
t0=$(date +%s.%N)
./oracle/_ref/c_p_np_aln -p 0 $F.fa > $F.mfa 2> $F.err
t1=$(date +%s.%N)
echo "reference c_p_np_aln N=$N L=$L threads=${OMP_NUM_THREADS:-all} wall $(awk "BEGIN{print $t1 - $t0}") s" | tee $F.time
