#!/bin/bash
# quickprobs C3 with the device MEA (MLP_MEA_DEVICE=1) against the host MEA,
# alternating, outputs compared (GPU box).
set -e -o pipefail
mkdir -p gpurun_out/qpdev
python3 -c "
import sys; sys.path.insert(0, '.')
from mlprobs_amd import synth
synth.write_fasta('gpurun_out/qpdev/c3.fa', synth.family(512, 400, 0.7, seed=11))
"
for mode in host dev host dev; do
  if [ $mode = dev ]; then export MLP_MEA_DEVICE=1; else unset MLP_MEA_DEVICE; fi
  t0=$(date +%s.%N)
  MLP_CLI_TIMES=1 timeout -k 10 120 ./mlprobs_amd/cli/quickprobs gpurun_out/qpdev/c3.fa > gpurun_out/qpdev/out_$mode.fa 2> gpurun_out/qpdev/err
  t1=$(date +%s.%N)
  echo "$mode wall $(awk "BEGIN{print $t1 - $t0}") s $(grep -E 'construction' gpurun_out/qpdev/err | tr '\n' ' ')" | tee -a gpurun_out/qpdev/summary.txt
  grep host gpurun_out/qpdev/err | tee -a gpurun_out/qpdev/summary.txt
done
cmp gpurun_out/qpdev/out_host.fa gpurun_out/qpdev/out_dev.fa && echo "outputs identical" | tee -a gpurun_out/qpdev/summary.txt
