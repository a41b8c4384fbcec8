#!/bin/bash
# VALU / SALU / LDS instruction counts per kernel of one C3 posterior step for
# library variants (tools/build_variants.py), one rocprofv3 PMC pass each (the
# counters in one pass: 4 SQ counters):
#   tools/valu_ab.sh base s1 ...  -> gpurun_out/valu_ab/<v>/ and summary.txt
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/valu_ab
mkdir -p $O
for v in "$@"; do
  if [ "$v" = base ]; then unset MLP_LIB_VARIANT; else export MLP_LIB_VARIANT=$v; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$v -o p \
      --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --no-qp --no-shards --relax 0 > $O/$v.log 2>&1 \
      || { tail -5 $O/$v.log; exit 1; }
  python3 tools/valu_ab_summary.py $O/$v $v | tee -a $O/summary.txt
done
