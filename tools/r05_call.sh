#!/bin/bash
# r05 GPU call: MEA with the row above rotating into lane 0 (no readlane): parity, timing, quickprobs A/B, CLI tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/mea_bench6; mkdir -p $O

timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "profile or mea" > $O/t_base.txt 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/base -o m -- python3 tools/mea_bench.py 20 > $O/summary.txt 2> $O/base.err &&
timeout -k 10 240 bash tools/r05_qp_ab.sh prev 2 > $O/qp.log 2>&1 &&
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_cli_gpu.py > $O/t_cli.txt 2>&1
rc=$?; tail -n 2 $O/t_base.txt $O/t_cli.txt; cat $O/summary.txt gpurun_out/qp_ab/summary.txt; exit $rc
