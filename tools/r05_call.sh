#!/bin/bash
# r05 GPU call: the npdo merge (all three models) at 5 waves, no spill: c_p_np_aln -p 1 A/B against HEAD, CLI tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/npm; mkdir -p $O
MODE=1 timeout -k 10 300 bash tools/r05_cli_ab.sh prev 3 > $O/cli.log 2>&1 &&
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_cli_gpu.py tests/test_gpu_parity.py -k "npdo or cli or nonprog" > $O/t.txt 2>&1
rc=$?; tail -n 2 $O/t.txt; cat gpurun_out/cli_ab/summary.txt; exit $rc
