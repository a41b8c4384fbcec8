#!/bin/bash
# r05 GPU call: quickprobs C3 posteriors at 16 GB, the partition function's sweeps joined before the merge only
# (MLP_EXP_LATEJOIN=1) against per-sweep joins (default for QuickProbs), alternating; QP parity tests under it
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/latejoin; mkdir -p $O
MLP_EXP_LATEJOIN=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "qp" > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
FA=tests/golden/config/c3_512x400_s11.fa
for k in 1 2 3; do for v in 0 1; do
  MLP_EXP_LATEJOIN=$v MLP_CLI_TIMES=1 timeout -k 10 120 mlprobs_amd/cli/quickprobs $FA > $O/q.msa 2> $O/e.txt || { tail -5 $O/e.txt; exit 1; }
  echo "latejoin $v qp run $k: $(grep -E '^\[stage\] (posteriors) ' $O/e.txt | tr '\n' ' ') $(cmp -s $O/q.msa tests/golden/config/c3_512x400_s11.qp.out && echo identical)" | tee -a $O/summary.txt
done; done
rm -f gpurun_out/variants/summary.txt
cd $GRAFT_REPO_ROOT
for v in 0 1 0 1; do MLP_EXP_LATEJOIN=$v timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --relax 0 --no-shards --steps 2 --warmup 1 2> /dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('latejoin $v qp posterior ms', round(d['quickprobs']['posterior_ms'],1))"; done
