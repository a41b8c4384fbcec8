set -e -o pipefail
O=gpurun_out/r01w; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "relax or qp" > $O/pytest.log 2>&1
timeout -k 10 150 python -u tools/relax_bench.py > $O/h2.log 2>&1
for v in h1 h3 h4; do
  MLP_LIB_VARIANT=$v timeout -k 10 150 python -u tools/relax_bench.py > $O/$v.log 2>&1
done
MLP_LIB_VARIANT=stats timeout -k 10 150 python -u tools/relax_bench.py 256 400 > $O/stats.log 2>&1
