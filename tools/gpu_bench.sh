#!/bin/bash
# The round's bench line (plain `python3 bench.py`, as the driver runs it) and
# the rocprofv3 kernel statistics of the bench's own kernels (the same bench
# under rocprofv3 with --no-e2e: the end-to-end legs are separate CLI
# processes and would mix their kernels into the summary).
#   tools/gpu_bench.sh TAG [bench args] -> gpurun_out/TAG/{bench.json,bench.log,bench_detail.json,prof_bench.json,stats/}
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-bench}; shift
O=gpurun_out/$TAG
mkdir -p $O
MLP_BENCH_DETAIL=$O/bench_detail.json timeout -k 10 900 python3 bench.py "$@" > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | tail -1 > $O/bench.json
grep '^\[bench' $O/bench.log
MLP_BENCH_DETAIL=$O/prof_detail.json timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o stats -- python3 bench.py --no-e2e --no-shards "$@" \
    > $O/prof_bench.log 2>&1 || { tail -30 $O/prof_bench.log; exit 1; }
grep '^{"metric"' $O/prof_bench.log | tail -1 > $O/prof_bench.json
