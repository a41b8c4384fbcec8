set -e -o pipefail
O=gpurun_out/r01fin; mkdir -p $O
timeout -k 10 500 python -u bench.py > $O/bench_plain.log 2>&1
bash tools/prof_bench.sh r01fin_prof
