#!/bin/bash
# Posterior-stage timing of the default build under environment settings:
#   tools/env_bench.sh "MLP_CHAIN_ROWS=1024" "MLP_CHAIN_ROWS=2048 X=1" ...
#   -> gpurun_out/envbench/summary.txt
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/envbench
mkdir -p $O
i=0
for spec in "$@"; do
  i=$((i + 1))
  timeout -k 10 300 env $spec python3 bench.py --no-cpu --no-e2e --no-qp --relax ${RELAX:-0} --steps 2 --warmup 1 > $O/$i.json 2> $O/$i.err || { tail -5 $O/$i.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('$O/$i.json'))
k=d['kernels_ms_per_step']; r=d.get('relax')
print('$spec', 'step %.1f ms' % d['ms_per_step'], ' '.join('%s %.1f' % (a, b) for a, b in k.items()),
      ('relax r1 %.1f ms' % r['round1']['kernel_ms']) if r else '')" | tee -a $O/summary.txt
done
