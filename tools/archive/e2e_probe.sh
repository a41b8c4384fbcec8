#!/bin/bash
# Where does a fresh c_p_np_aln process spend its time at C2 / C3 (GPU box)?
#   tools/e2e_probe.sh   -> gpurun_out/e2e/*
# 1. hipMalloc + first touch of large scratch in fresh processes, back to back
#    (does a process wait for the memory the previous one released?)
# 2. c_p_np_aln -p 0 at C2 then C3 (stage times), then C3 with other scratch budgets
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/e2e
mkdir -p $O
F2=tests/golden/config/c2_128x256_s11.fa
F3=tests/golden/config/c3_512x400_s11.fa
CLI=./mlprobs_amd/cli/c_p_np_aln
run() {  # tag, env..., -- args
  local tag=$1; shift
  local t0=$(date +%s.%N)
  timeout -k 10 120 env "$@" > $O/$tag.out 2> $O/$tag.err
  local rc=$?
  local t1=$(date +%s.%N)
  echo "$tag rc=$rc wall $(awk "BEGIN{print $t1 - $t0}")" | tee -a $O/summary.txt
  grep '^\[' $O/$tag.err | tee -a $O/summary.txt
  return $rc
}
timeout -k 10 60 tools/probe/alloc_probe 32 | tee -a $O/summary.txt || exit 1
timeout -k 10 60 tools/probe/alloc_probe 32 | tee -a $O/summary.txt || exit 1
timeout -k 10 60 tools/probe/alloc_probe 1 4 16 | tee -a $O/summary.txt || exit 1
run c2_a MLP_CLI_TIMES=1 $CLI -p 0 $F2 || exit 1
run c3_a MLP_CLI_TIMES=1 $CLI -p 0 $F3 || exit 1
run c3_b MLP_CLI_TIMES=1 $CLI -p 0 $F3 || exit 1
sleep 5
run c3_s8 MLP_CLI_TIMES=1 MLP_SCRATCH_GB=8 $CLI -p 0 $F3 || exit 1
run c3_s4 MLP_CLI_TIMES=1 MLP_SCRATCH_GB=4 $CLI -p 0 $F3 || exit 1
run c3_s64 MLP_CLI_TIMES=1 MLP_SCRATCH_GB=64 $CLI -p 0 $F3 || exit 1
run c3_s8b MLP_CLI_TIMES=1 MLP_SCRATCH_GB=8 $CLI -p 0 $F3 || exit 1
run c2_b MLP_CLI_TIMES=1 $CLI -p 0 $F2 || exit 1
run c2_s2 MLP_CLI_TIMES=1 MLP_SCRATCH_GB=2 $CLI -p 0 $F2 || exit 1
echo done
