#!/bin/bash
# r05 GPU call: partition-function sweeps at wave priority 1 (variant pfprio) -- c_p_np_aln C3 -p 0 posteriors
# at 16 GB and quickprobs C3 against the default, alternating; then the bench step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pfprio; mkdir -p $O
mkdir -p /tmp/v_pfprio && ln -sf $PWD/mlprobs_amd/lib/libmlpgpu_pfprio.so /tmp/v_pfprio/libmlpgpu.so
FA=tests/golden/config/c3_512x400_s11.fa
for k in 1 2 3; do for v in base pfprio; do
  LP=; [ $v = pfprio ] && LP=/tmp/v_pfprio
  LD_LIBRARY_PATH=$LP MLP_CLI_TIMES=1 timeout -k 10 120 mlprobs_amd/cli/c_p_np_aln -p 0 $FA > $O/o.msa 2> $O/e.txt || { tail -5 $O/e.txt; exit 1; }
  echo "$v -p 0 run $k: $(grep -E '^\[stage\] (posteriors) ' $O/e.txt | tr '\n' ' ') $(cmp -s $O/o.msa tests/golden/config/c3_512x400_s11.p_0.out && echo identical)" | tee -a $O/summary.txt
  LD_LIBRARY_PATH=$LP MLP_CLI_TIMES=1 timeout -k 10 120 mlprobs_amd/cli/quickprobs $FA > $O/q.msa 2> $O/e.txt || { tail -5 $O/e.txt; exit 1; }
  echo "$v qp run $k: $(grep -E '^\[stage\] (posteriors) ' $O/e.txt | tr '\n' ' ') $(cmp -s $O/q.msa tests/golden/config/c3_512x400_s11.qp.out && echo identical)" | tee -a $O/summary.txt
done; done
rm -f gpurun_out/variants/summary.txt
bash tools/variant_bench.sh base pfprio base pfprio
