set -e -o pipefail
O=gpurun_out/r01u; mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
