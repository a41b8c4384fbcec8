#!/bin/bash
# r05 GPU call: quickprobs device-MEA floor 50k -- CLI, heavy-family and pipeline GPU tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/meamin2; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_cli_gpu.py tests/test_heavy_gpu.py tests/test_pipeline_gpu.py > $O/t.txt 2>&1
rc=$?; tail -n 2 $O/t.txt; exit $rc
