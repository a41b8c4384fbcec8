set -e -o pipefail
O=gpurun_out/r01p; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "relax" > $O/pytest_relax.log 2>&1
timeout -k 10 200 python -u tools/relax_bench.py > $O/relax.log 2>&1
