#!/bin/bash
# The quickprobs drop-in on C3 with experiment builds of the library
# (tools/build_variants.py; the CLI's RUNPATH yields to LD_LIBRARY_PATH):
# stage split per run, output bytes against the default build's.
#   tools/qp_variant_ab.sh base v1 v2 ... -> gpurun_out/qp_variant_ab/summary.txt
export TMPDIR=/tmp
O=gpurun_out/qp_variant_ab
mkdir -p $O
FA=tests/golden/config/c3_512x400_s11.fa
CLI=mlprobs_amd/cli/quickprobs
for rep in 1 2; do for v in "$@"; do
  if [ "$v" = base ]; then unset LD_LIBRARY_PATH; else
    mkdir -p /tmp/mlpvar_$v && cp mlprobs_amd/lib/libmlpgpu_$v.so /tmp/mlpvar_$v/libmlpgpu.so && export LD_LIBRARY_PATH=/tmp/mlpvar_$v; fi
  MLP_CLI_TIMES=1 timeout -k 10 120 $CLI $FA > $O/out_$v.fa 2> $O/err_$v.txt || { tail -5 $O/err_$v.txt; exit 1; }
  same=$(cmp -s $O/out_$v.fa $O/out_base.fa 2>/dev/null && echo same-bytes)
  echo "$v run $rep: $(grep -E '^\[stage\] (posteriors|consistency|construction)' $O/err_$v.txt | tr '\n' ' ') $(grep -oE 'MEA [0-9.]+ s' $O/err_$v.txt) $same" | tee -a $O/summary.txt
done; done
