#!/bin/bash
# Relaxation tile classes at C3: round 2 (tiles fit half the LDS: two
# workgroups per CU, 8 waves per SIMD) against the same round forced into the
# one-workgroup class (MLP_RELAX_ONECLASS=1: 4 waves per SIMD, register
# prefetch); then the QuickProbs C3 drop-in's host/device time split.
#   tools/relax_class_ab.sh TAG -> gpurun_out/TAG/
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-relaxab}
O=gpurun_out/$TAG
mkdir -p $O
for mode in two one; do
  if [ $mode = one ]; then export MLP_RELAX_ONECLASS=1; else unset MLP_RELAX_ONECLASS; fi
  MLP_PLAN_LOG=1 timeout -k 10 300 python3 bench.py --no-e2e --no-cpu --no-qp --relax 2 --steps 1 --warmup 0 \
      > $O/b_$mode.log 2>&1 || { tail -20 $O/b_$mode.log; exit 1; }
  grep "relax plan" $O/b_$mode.log
  python3 -c "
import json
d=json.loads([l for l in open('$O/b_$mode.log') if l.startswith('{\"metric')][-1])
for r in d['relax']['per_round']: print('$mode', r['nnz_in'], round(r['seconds'],3), {k: round(v,1) for k,v in r['kernels_ms'].items()})
"
done
unset MLP_RELAX_ONECLASS
python3 -c "
import sys; sys.path.insert(0, '.')
from mlprobs_amd import synth
synth.write_fasta('$O/c3.fa', synth.family(512, 400, 0.7, seed=11))
" || exit 1
t0=$(date +%s.%N)
MLP_CLI_TIMES=1 timeout -k 10 120 ./mlprobs_amd/cli/quickprobs $O/c3.fa > $O/qp.out 2> $O/qp.err || { cat $O/qp.err; exit 1; }
echo "quickprobs C3 wall $(awk "BEGIN{print $(date +%s.%N) - $t0}") s"
cat $O/qp.err
