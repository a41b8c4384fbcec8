#!/bin/bash
# Small-class relaxation tiles with in-HBM images on oversize z's: the relax
# parity tests, then C3 rounds 1-2 (and the QuickProbs consistency round) per
# MLP_RELAX_GLOBAL_Z value ("default" = unset; 0 = the one-workgroup class
# for such outputs).   tools/relax_hbm_ab.sh TAG VALUES... -> gpurun_out/TAG/
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-relaxhbm}; shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "relax" > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
tail -2 $O/test.log
for gz in "$@"; do
  if [ $gz = default ]; then unset MLP_RELAX_GLOBAL_Z; else export MLP_RELAX_GLOBAL_Z=$gz; fi
  MLP_PLAN_LOG=1 timeout -k 10 300 python3 bench.py --no-e2e --no-cpu --relax 2 --steps 1 --warmup 0 \
      > $O/b_$gz.log 2>&1 || { tail -20 $O/b_$gz.log; exit 1; }
  grep "relax plan" $O/b_$gz.log
  python3 -c "
import json
d=json.loads([l for l in open('$O/b_$gz.log') if l.startswith('{\"metric')][-1])
for r in d['relax']['per_round']: print('glob $gz', r['nnz_in'], round(r['seconds'],3), {k: round(v,1) for k,v in r['kernels_ms'].items()})
print('glob $gz quickprobs consistency round', round(d['quickprobs']['consistency_round_s'],3))
"
done
