#!/bin/bash
# r05 GPU call: deferred batch finish (batch b+1's sweeps launched before batch b's host part and compaction)
# -- posterior/totals/config/shard parity, the CLI tests, then c_p_np_aln C3 -p 0 posteriors at 16 GB against
# MLP_DEFER_FINISH=0 and the bench step, alternating
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/defer; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_totals.py tests/test_gpu_configs.py tests/test_gpu_shards.py tests/test_cli_gpu.py > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
FA=tests/golden/config/c3_512x400_s11.fa
for k in 1 2 3; do for v in 0 1; do
  MLP_DEFER_FINISH=$v MLP_CLI_TIMES=1 timeout -k 10 120 mlprobs_amd/cli/c_p_np_aln -p 0 $FA > $O/o.msa 2> $O/e.txt || { tail -5 $O/e.txt; exit 1; }
  echo "defer $v run $k: $(grep -E '^\[stage\] (posteriors) ' $O/e.txt | tr '\n' ' ') $(cmp -s $O/o.msa tests/golden/config/c3_512x400_s11.p_0.out && echo identical)" | tee -a $O/summary.txt
done; done
rm -f gpurun_out/variants/summary.txt
bash tools/variant_bench.sh base:MLP_DEFER_FINISH=0 base base:MLP_DEFER_FINISH=0 base
