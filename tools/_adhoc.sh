set -e -o pipefail
O=gpurun_out/r01t; mkdir -p $O
python3 -c "
import sys; sys.path.insert(0, '.')
from mlprobs_amd import synth
synth.write_fasta('$O/c3.fa', synth.family(512, 400, 0.7, seed=11))
"
for gb in 64 64 16 24 32 16; do
  t0=$(date +%s.%N)
  MLP_SCRATCH_GB=$gb MLP_CLI_TIMES=1 timeout -k 10 120 ./mlprobs_amd/cli/c_p_np_aln -p 0 $O/c3.fa > $O/cp_$gb.fa 2> $O/cp_$gb.err
  t1=$(date +%s.%N)
  echo "c_p_np_aln scratch $gb GB: wall $(awk "BEGIN{print $t1 - $t0}") s $(grep posteriors $O/cp_$gb.err)" >> $O/scan.log
done
md5sum $O/cp_*.fa >> $O/scan.log
t0=$(date +%s.%N)
MLP_CLI_TIMES=1 timeout -k 10 120 ./mlprobs_amd/cli/quickprobs $O/c3.fa > $O/qp.fa 2> $O/qp.err
t1=$(date +%s.%N)
echo "quickprobs wall $(awk "BEGIN{print $t1 - $t0}") s" >> $O/scan.log
cat $O/qp.err >> $O/scan.log
