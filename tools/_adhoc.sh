set -e -o pipefail
O=gpurun_out/r01w3; mkdir -p $O
MLP_LIB_VARIANT=timing timeout -k 10 150 python -u tools/relax_bench.py > $O/timing.log 2>&1
