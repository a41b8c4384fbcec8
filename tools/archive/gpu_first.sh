#!/bin/bash
# Round-3 first pass: HBM stream peak, the -m gpu suite, smoke, one bench.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-first}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 120 tools/probe/hbm_stream 8 10 > $O/stream.json 2> $O/stream.err || { cat $O/stream.err; exit 1; }
cat $O/stream.json
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
grep '^{"metric"' $O/bench.log | tail -1 > $O/bench.json
echo done
