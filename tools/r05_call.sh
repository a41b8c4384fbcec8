#!/bin/bash
# r05 GPU call: new defaults (forward-chain totals beside the backward sweeps at wave priority 3, batch
# planning calibrated to the planned chains, balanced batches) -- GPU suite, then c_p_np_aln C3 -p 0 / -p 1 and
# quickprobs C3 against HEAD's library, alternating
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/newdef; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
mkdir -p /tmp/v_head && ln -sf $PWD/mlprobs_amd/lib/libmlpgpu_head.so /tmp/v_head/libmlpgpu.so
FA=tests/golden/config/c3_512x400_s11.fa
for k in 1 2 3; do for v in head new; do
  LP=; [ $v = head ] && LP=/tmp/v_head
  LD_LIBRARY_PATH=$LP MLP_CLI_TIMES=1 timeout -k 10 120 mlprobs_amd/cli/c_p_np_aln -p 0 $FA > $O/o.msa 2> $O/e.txt || { tail -5 $O/e.txt; exit 1; }
  echo "$v -p 0 run $k: $(grep -E '^\[stage\] (posteriors|consistency) ' $O/e.txt | tr '\n' ' ') $(cmp -s $O/o.msa tests/golden/config/c3_512x400_s11.p_0.out && echo identical)" | tee -a $O/summary.txt
  LD_LIBRARY_PATH=$LP MLP_CLI_TIMES=1 timeout -k 10 120 mlprobs_amd/cli/quickprobs $FA > $O/q.msa 2> $O/e.txt || { tail -5 $O/e.txt; exit 1; }
  echo "$v qp run $k: $(grep -E '^\[stage\] (posteriors|consistency) ' $O/e.txt | tr '\n' ' ') $(cmp -s $O/q.msa tests/golden/config/c3_512x400_s11.qp.out && echo identical)" | tee -a $O/summary.txt
done; done
