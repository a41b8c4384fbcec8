set -e -o pipefail
O=gpurun_out/r01s4; mkdir -p $O
timeout -k 10 150 python -u tools/relax_bench.py > $O/relax.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
