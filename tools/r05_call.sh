#!/bin/bash
# r05 GPU call: after the device-MEA mask fix and the deferred-matrix pinned buffer -- MEA/profile parity tests,
# every CLI GPU test, and C2 -p 1 stage times (teardown) at the default floor
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/p1f; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "mea or profile" > $O/t1.txt 2>&1 || { tail -30 $O/t1.txt; exit 1; }
tail -1 $O/t1.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_cli_gpu.py > $O/t2.txt 2>&1 || { tail -30 $O/t2.txt; exit 1; }
tail -1 $O/t2.txt
c=c2_128x256_s11; FA=tests/golden/config/$c.fa
for k in 1 2; do
  MLP_SRAND_TIME=1700000000 MLP_CLI_TIMES=1 timeout -k 10 120 mlprobs_amd/cli/c_p_np_aln -p 1 $FA > $O/$c.msa 2> $O/$c.txt || { tail -5 $O/$c.txt; exit 1; }
  echo "$c -p 1 run $k: $(grep -E '^\[stage\] (refinement|context teardown)' $O/$c.txt | tr '\n' ' ') $(cmp -s $O/$c.msa tests/golden/config/$c.p_1.out && echo identical-to-ref)"
done
