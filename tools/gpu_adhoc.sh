#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/np2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "profile_posterior_on_gpu or pf_long_double or cli_progressive or cli_config or npdo or test_real_families" > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
timeout -k 10 300 python3 bench.py --no-cpu --no-qp --relax 0 --steps 1 --warmup 0 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json'))
for k,v in d['e2e'].items(): print(k, round(v['seconds'],3), {a: round(b,3) for a,b in v['stages_s'].items()})"
