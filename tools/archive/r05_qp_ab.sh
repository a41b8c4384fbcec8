#!/bin/bash
# quickprobs drop-in on C3: the current library (new) against a variant build (LD_LIBRARY_PATH), alternating,
# stage times, outputs compared with each other and with the first run's
#   tools/r05_qp_ab.sh VARIANT [runs] -> gpurun_out/qp_ab/summary.txt
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/qp_ab
mkdir -p $O
V=$1; N=${2:-3}
mkdir -p /tmp/v_$V && ln -sf $PWD/mlprobs_amd/lib/libmlpgpu_$V.so /tmp/v_$V/libmlpgpu.so
FA=tests/golden/config/c3_512x400_s11.fa
for k in $(seq $N); do for v in new $V; do
  LP=; [ $v != new ] && LP=/tmp/v_$V
  LD_LIBRARY_PATH=$LP MLP_CLI_TIMES=1 MLP_LOG_PROFILE=1 timeout -k 10 120 mlprobs_amd/cli/quickprobs $FA > $O/out_$v.fa 2> $O/err_$v.txt || { tail -5 $O/err_$v.txt; exit 1; }
  [ -f $O/ref.fa ] || cp $O/out_$v.fa $O/ref.fa
  echo "$v run $k: $(grep -E '^\[stage\] (posteriors|consistency|construction \+ refinement|output)|^\[profile posterior\]' $O/err_$v.txt | tr '\n' ' ') $(cmp -s $O/out_$v.fa $O/ref.fa && echo same-output)" | tee -a $O/summary.txt
done; done
