set -e -o pipefail
O=gpurun_out/r01s7; mkdir -p $O
for r in 1 2; do
for v in m4 m6 m7; do
  MLP_LIB_VARIANT=$v timeout -k 10 300 python -u bench.py --no-e2e --no-qp --relax 0 --no-cpu --steps 5 > $O/$v$r.log 2>&1
done
done
