#!/bin/bash
# r05 GPU call: LOOKUP row as a byte offset (no clamp, no shift; MLP_LOOKUP_BYTEOFF) -- parity under the variant, then posterior-step A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/bo; mkdir -p $O
MLP_LIB_VARIANT=bo timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_totals.py tests/test_gpu_configs.py > $O/t_bo.txt 2>&1 &&
RELAX=0 timeout -k 10 400 bash tools/variant_bench.sh base bo base bo > $O/vb.log 2>&1
rc=$?; tail -n 2 $O/t_bo.txt; cat gpurun_out/variants/summary.txt; exit $rc
