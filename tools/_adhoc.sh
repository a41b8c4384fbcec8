set -e -o pipefail
O=gpurun_out/r01tp; mkdir -p $O
for rep in 1 2; do
for v in base tp4 tp16; do
  if [ $v = base ]; then unset MLP_LIB_VARIANT; else export MLP_LIB_VARIANT=$v; fi
  timeout -k 10 300 python -u bench.py --no-e2e --no-qp --relax 0 --no-cpu --steps 5 > $O/$v$rep.log 2>&1
done
done
MLP_LIB_VARIANT=tp4 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest4.log 2>&1
MLP_LIB_VARIANT=tp16 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest16.log 2>&1
