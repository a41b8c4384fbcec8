#!/bin/bash
# PMC passes over one C3 relaxation round (tools/relax_bench.py), relaxation
# kernels only.  Run on the GPU box from the repo root.
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/rpmc}
ARGS=${2:-512 400}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex relax -d $OUT/p1 -o p --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU -- python3 tools/relax_bench.py $ARGS > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex relax -d $OUT/p2 -o p --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU -- python3 tools/relax_bench.py $ARGS > $OUT/p2.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex relax -d $OUT/p3 -o p --pmc FETCH_SIZE -- python3 tools/relax_bench.py $ARGS > $OUT/p3.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex relax -d $OUT/p4 -o p --pmc TCC_HIT_sum TCC_MISS_sum -- python3 tools/relax_bench.py $ARGS > $OUT/p4.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex relax -d $OUT/p5 -o p --pmc TCC_REQ_sum TCC_EA0_RDREQ_sum -- python3 tools/relax_bench.py $ARGS > $OUT/p5.log 2>&1
