#!/bin/bash
# Kernel trace of the C3 posterior stage under environment settings:
#   tools/trace_cfg.sh NAME "ENV=.. ENV=.." ... -> gpurun_out/trace/NAME/*kernel_trace.csv
set -o pipefail
export TMPDIR=/tmp
while [ $# -ge 2 ]; do
  name=$1; spec=$2; shift 2
  O=gpurun_out/trace/$name
  mkdir -p $O
  env $spec timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- \
      python3 bench.py --no-cpu --no-e2e --no-qp --relax 0 --steps 1 --warmup 0 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
  f=$(find $O -name '*kernel_trace.csv' | head -1)
  python3 tools/trace_summary.py "$f" | tee $O/summary.txt
done
