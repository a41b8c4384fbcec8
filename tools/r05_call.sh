#!/bin/bash
# r05 GPU call: profile posterior adds eight pairs per LDS round trip: parity, quickprobs A/B against HEAD, CLI tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pp8; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "profile or mea" > $O/t_base.txt 2>&1 &&
timeout -k 10 240 bash tools/r05_qp_ab.sh prev 3 > $O/qp.log 2>&1 &&
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_cli_gpu.py > $O/t_cli.txt 2>&1
rc=$?; tail -n 2 $O/t_base.txt $O/t_cli.txt; cat gpurun_out/qp_ab/summary.txt; grep -h "\[host\]" gpurun_out/qp_ab/err_new.txt; exit $rc
