#!/bin/bash
# r05 GPU call: bench step, lane fold kernels at wave priority 3 (variant lfprio), with and without the lane
# fold's forward half beside the backward sweeps (MLP_LF_BESIDE=1), against the default
set -o pipefail
export TMPDIR=/tmp
rm -f gpurun_out/variants/summary.txt
bash tools/variant_bench.sh base lfprio lfprio:MLP_LF_BESIDE=1 base:MLP_LF_BESIDE=1 base lfprio lfprio:MLP_LF_BESIDE=1 base:MLP_LF_BESIDE=1
