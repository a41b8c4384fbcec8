#!/bin/bash
# Where the progressive/refinement stages spend their time (GPU box):
#   tools/refine_probe.sh -> gpurun_out/refine/summary.txt
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/refine
mkdir -p $O
F2=tests/golden/config/c2_128x256_s11.fa
F3=tests/golden/config/c3_512x400_s11.fa
run() {  # tag, command...
  local tag=$1; shift
  local t0=$(date +%s.%N)
  timeout -k 10 120 env MLP_CLI_TIMES=1 MLP_PROFILE_TIMES=1 "$@" > $O/$tag.out 2> $O/$tag.err
  local rc=$?
  echo "$tag rc=$rc wall $(awk "BEGIN{print $(date +%s.%N) - $t0}")" | tee -a $O/summary.txt
  grep '^\[' $O/$tag.err | tee -a $O/summary.txt
  return $rc
}
run c2_p0 ./mlprobs_amd/cli/c_p_np_aln -p 0 $F2 || exit 1
run c2_p1 env MLP_SRAND_TIME=1 ./mlprobs_amd/cli/c_p_np_aln -p 1 $F2 || exit 1
run qp_c2 ./mlprobs_amd/cli/quickprobs $F2 || exit 1
run qp_c3 ./mlprobs_amd/cli/quickprobs $F3 || exit 1
