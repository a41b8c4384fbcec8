set -e -o pipefail
O=gpurun_out/r01y5; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_cli_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k real > $O/pytest.log 2>&1
