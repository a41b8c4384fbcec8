#!/bin/bash
# PMC passes over the posterior stage's k_local_totals only (GPU box, repo root).
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/tpmc}
mkdir -p $OUT
ARGS="--steps 1 --warmup 0 --no-cpu --no-e2e --no-qp --no-shards --relax 0"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex local_totals -d $OUT/p1 -o p --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM -- python3 bench.py $ARGS > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex local_totals -d $OUT/p2 -o p --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -- python3 bench.py $ARGS > $OUT/p2.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex local_totals -d $OUT/p3 -o p --pmc FETCH_SIZE -- python3 bench.py $ARGS > $OUT/p3.log 2>&1
