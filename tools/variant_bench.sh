#!/bin/bash
# Posterior-stage timing of experiment builds (tools/build_variants.py) on the
# GPU box: tools/variant_bench.sh base v1 v2 ... -> gpurun_out/variants/summary.txt
# An entry may carry one environment setting: base:MLP_TEST_TOT_LANEFOLD=1
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/variants
mkdir -p $O
for spec in "$@"; do
  v=${spec%%:*}
  if [ "$v" = base ]; then unset MLP_LIB_VARIANT; else export MLP_LIB_VARIANT=$v; fi
  setting=""; [ "$spec" != "$v" ] && setting=${spec#*:}
  v=$(echo "$spec" | tr ':=' '__')
  timeout -k 10 300 env $setting python3 bench.py --no-cpu --no-e2e --no-qp --relax ${RELAX:-0} --no-shards --steps 2 --warmup 1 > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('$O/$v.json'))
k=d['kernels_ms_per_step']; r=d.get('relax')
print('$v', 'step %.1f ms' % d['ms_per_step'], ' '.join('%s %.1f' % (a, b) for a, b in k.items()),
      ('relax r1 %.1f ms' % r['round1']['kernel_ms']) if r else '')" | tee -a $O/summary.txt
done
