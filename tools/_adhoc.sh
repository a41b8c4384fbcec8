set -e -o pipefail
O=gpurun_out/r01o; mkdir -p $O
MLP_LIB_VARIANT=nostage timeout -k 10 200 python -u tools/relax_bench.py > $O/relax_nostage.log 2>&1
