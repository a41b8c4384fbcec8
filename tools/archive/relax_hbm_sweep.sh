#!/bin/bash
# C3 round 1 with every small-class output allowed in-HBM images
# (MLP_RELAX_GLOBAL_Z=512), over staging sizes and pass limits; phase log.
#   tools/relax_hbm_sweep.sh TAG "SMALL_KB:SPLIT_Z" ... -> gpurun_out/TAG/
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-relaxsweep}; shift
O=gpurun_out/$TAG
mkdir -p $O
for cfg in "$@"; do
  kb=${cfg%%:*}; sz=${cfg##*:}
  env MLP_RELAX_GLOBAL_Z=512 MLP_RELAX_SMALL_KB=$kb MLP_RELAX_SPLIT_Z=$sz MLP_PLAN_LOG=1 MLP_RELAX_LOG=1 \
      timeout -k 10 300 python3 bench.py --no-e2e --no-cpu --no-qp --relax 1 --steps 1 --warmup 0 \
      > $O/b_${kb}_$sz.log 2>&1 || { tail -20 $O/b_${kb}_$sz.log; exit 1; }
  echo "== SMALL_KB $kb SPLIT_Z $sz"
  grep -E "relax plan|\[relax\]" $O/b_${kb}_$sz.log | head -12
done
