#!/bin/bash
# quickprobs C3 twice per MEA setting (single-thread SIMD strips vs threaded),
# the first run of each pair absorbing the device's memory clearing.
set -e -o pipefail
mkdir -p gpurun_out/qpab
python3 -c "
import sys; sys.path.insert(0, '.')
from mlprobs_amd import synth
synth.write_fasta('gpurun_out/qpab/c3.fa', synth.family(512, 400, 0.7, seed=11))
"
for setting in 1000000000000 1000000 1000000000000 1000000; do
  for rep in 1 2; do
    MLP_MEA_THREAD_MIN=$setting MLP_CLI_TIMES=1 timeout -k 10 120 ./mlprobs_amd/cli/quickprobs gpurun_out/qpab/c3.fa > gpurun_out/qpab/out_$setting.fa 2> gpurun_out/qpab/err
    echo "thread_min=$setting rep=$rep $(grep -E 'posteriors [0-9]|construction' gpurun_out/qpab/err | tr '\n' ' ')" | tee -a gpurun_out/qpab/summary.txt
    grep host gpurun_out/qpab/err | tee -a gpurun_out/qpab/summary.txt
  done
done
cmp gpurun_out/qpab/out_1000000.fa gpurun_out/qpab/out_1000000000000.fa && echo "outputs identical" | tee -a gpurun_out/qpab/summary.txt
