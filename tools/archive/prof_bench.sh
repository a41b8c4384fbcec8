#!/bin/bash
# The round's bench line and its rocprofv3 kernel statistics from ONE command
# (so bench's HIP-event launch averages and rocprof's agree), on the GPU box:
#   tools/prof_bench.sh TAG  -> gpurun_out/TAG/{bench.json,stats/...}
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-prof}
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o stats -- python3 bench.py > $O/bench.log 2>&1
grep '^{"metric"' $O/bench.log | tail -1 > $O/bench.json
