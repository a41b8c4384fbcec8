#!/bin/bash
# r05 GPU call: quickprobs A/B of k_profile_post (run-ahead extents) + the CLI / pipeline GPU tests
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 bash tools/r05_qp_ab.sh prev 3 > gpurun_out/qp_ab.log 2>&1 &&
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_cli_gpu.py tests/test_pipeline_gpu.py > gpurun_out/t_cli.txt 2>&1
rc=$?; tail -3 gpurun_out/t_cli.txt; cat gpurun_out/qp_ab/summary.txt; exit $rc
