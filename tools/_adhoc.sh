set -e -o pipefail
O=gpurun_out/r01s6; mkdir -p $O
for r in 1 2; do
for v in w4 w6; do
  MLP_LIB_VARIANT=$v timeout -k 10 300 python -u bench.py --no-e2e --no-qp --relax 0 --no-cpu --steps 5 > $O/$v$r.log 2>&1
done
done
MLP_LIB_VARIANT=w6 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
