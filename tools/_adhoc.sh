set -e -o pipefail
O=gpurun_out/r01y; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 200 python -u tools/relax_bench.py > $O/relax.log 2>&1
