set -e -o pipefail
O=gpurun_out/r01z2; mkdir -p $O
timeout -k 10 150 python -u tools/relax_bench.py > $O/base.log 2>&1
MLP_LIB_VARIANT=t512 timeout -k 10 150 python -u tools/relax_bench.py > $O/t512.log 2>&1
MLP_LIB_VARIANT=t512 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "relax or qp" > $O/pytest.log 2>&1
