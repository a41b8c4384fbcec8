set -e -o pipefail
O=gpurun_out/r01pq; mkdir -p $O
timeout -k 10 300 bash tools/qp_cli_time.sh 512 400 > $O/qp_c3.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k profile > $O/pytest_prof.log 2>&1
timeout -k 10 900 python -u -m pytest tests/test_cli_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_cli.log 2>&1
