set -e -o pipefail
O=gpurun_out/r01sw; mkdir -p $O
timeout -k 10 1100 python -u tools/parity_sweep.py $O/sweep.txt 8 > $O/sweep.log 2>&1
