set -e -o pipefail
O=gpurun_out/r01cr3; mkdir -p $O
for rep in 1 2; do
  MLP_CHAIN_ROWS=1282 timeout -k 10 300 python -u bench.py --no-e2e --no-qp --relax 0 --no-cpu --steps 5 > $O/old$rep.log 2>&1
  timeout -k 10 300 python -u bench.py --no-e2e --no-qp --relax 0 --no-cpu --steps 5 > $O/new$rep.log 2>&1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
