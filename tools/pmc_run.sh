#!/bin/bash
# PMC passes for the posterior stage (run on the GPU box from the repo root).
# Counters are collected in separate passes with --kernel-trace only, as the
# MI355X guide prescribes (FETCH_SIZE and WRITE_SIZE cannot share a pass).
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc}
ARGS=${2:---steps 1 --warmup 0 --no-cpu}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/p1 -o p1 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS -- python3 bench.py $ARGS > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/p2 -o p2 --pmc FETCH_SIZE -- python3 bench.py $ARGS > $OUT/p2.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/p3 -o p3 --pmc WRITE_SIZE -- python3 bench.py $ARGS > $OUT/p3.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o stats -- python3 bench.py $ARGS > $OUT/stats.log 2>&1
