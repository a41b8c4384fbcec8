#!/bin/bash
# c_p_np_aln -p 0 drop-in on C3: the current library (new) against a variant build (LD_LIBRARY_PATH), alternating;
# stage times, output compared with the reference CLI's
#   tools/r05_cli_ab.sh VARIANT [runs] -> gpurun_out/cli_ab/summary.txt
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/cli_ab
mkdir -p $O
V=$1; N=${2:-3}
mkdir -p /tmp/v_$V && ln -sf $PWD/mlprobs_amd/lib/libmlpgpu_$V.so /tmp/v_$V/libmlpgpu.so
FA=tests/golden/config/c3_512x400_s11.fa
for k in $(seq $N); do for v in new $V; do
  LP=; [ $v != new ] && LP=/tmp/v_$V
  LD_LIBRARY_PATH=$LP MLP_CLI_TIMES=1 timeout -k 10 120 mlprobs_amd/cli/c_p_np_aln -p ${MODE:-0} $FA > $O/out_$v.msa 2> $O/err_$v.txt || { tail -5 $O/err_$v.txt; exit 1; }
  echo "$v run $k: $(grep -E '^\[stage\] (posteriors|consistency) ' $O/err_$v.txt | tr '\n' ' ') $(cmp -s $O/out_$v.msa tests/golden/config/c3_512x400_s11.p_${MODE:-0}.out && echo identical)" | tee -a $O/summary.txt
done; done
