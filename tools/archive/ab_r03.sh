#!/bin/bash
# Round-3 A/B pass on the GPU box:
#   1. posterior stage with the side stream joined after each sweep (MLP_JOIN=0),
#      joined before the merge (1) and as per-model chains (2), alternating;
#   2. quickprobs C3 end to end with the host MEA and the device MEA
#      (MLP_MEA_DEVICE=1), alternating, outputs compared;
#   3. the allocation probe sequence (tools/probe/alloc_seq.sh).
#   tools/ab_r03.sh [parts...] -> gpurun_out/ab/summary.txt
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
PARTS=${*:-"join mea alloc"}
F3=tests/golden/config/c3_512x400_s11.fa
for part in $PARTS; do
case $part in
join)
  for rep in 1 2; do
    for j in 0 1 2; do
      MLP_JOIN=$j timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --no-qp --relax 0 --no-shards --steps 3 --warmup 1 \
        > $O/join$j.json 2> $O/join$j.err || { tail -5 $O/join$j.err; exit 1; }
      python3 -c "
import json; d=json.load(open('$O/join$j.json'))
k=d['kernels_ms_per_step']
print('MLP_JOIN=$j', 'step %.1f ms' % d['ms_per_step'], ' '.join('%s %.1f' % (a, b) for a, b in k.items()))" | tee -a $O/summary.txt
    done
  done ;;
mea)
  for rep in 1 2; do
    for m in 0 1; do
      t0=$(date +%s.%N)
      MLP_MEA_DEVICE=$m MLP_CLI_TIMES=1 timeout -k 10 120 ./mlprobs_amd/cli/quickprobs $F3 > $O/qp$m.out 2> $O/qp$m.err || { tail -5 $O/qp$m.err; exit 1; }
      t1=$(date +%s.%N)
      echo "quickprobs C3 MLP_MEA_DEVICE=$m wall $(awk "BEGIN{print $t1 - $t0}")" | tee -a $O/summary.txt
      grep -E 'construction|\[host\]|posteriors' $O/qp$m.err | tee -a $O/summary.txt
    done
    cmp $O/qp0.out $O/qp1.out && echo "quickprobs C3 host / device MEA outputs identical" | tee -a $O/summary.txt
  done ;;
jointest)
  for j in 1 2; do
    MLP_JOIN=$j timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
      > $O/jointest$j.log 2>&1 || { tail -20 $O/jointest$j.log; exit 1; }
    echo "MLP_JOIN=$j parity tests: $(tail -1 $O/jointest$j.log)" | tee -a $O/summary.txt
  done ;;
cap)
  # c_p_np_aln C3 -p 0 back to back at several scratch caps, after a process
  # that held ~150 GB (the bench's posterior stage)
  for cap in ${CAPS:-16 24 32}; do
    timeout -k 10 200 python3 bench.py --no-cpu --no-e2e --no-qp --relax 0 --no-shards --steps 1 --warmup 0 > /dev/null 2>&1 || exit 1
    for rep in 1 2 3 4; do
      t0=$(date +%s.%N)
      MLP_SCRATCH_GB=$cap MLP_CLI_TIMES=1 timeout -k 10 120 ./mlprobs_amd/cli/c_p_np_aln -p 0 $F3 > $O/cap.out 2> $O/cap.err || { tail -5 $O/cap.err; exit 1; }
      t1=$(date +%s.%N)
      echo "C3 -p 0 scratch $cap GB run $rep wall $(awk "BEGIN{print $t1 - $t0}") $(grep -E '^\[stage\] posteriors' $O/cap.err)" | tee -a $O/summary.txt
    done
    cmp -s $O/cap.out tests/golden/config/c3_512x400_s11.p_0.out && echo "C3 -p 0 output = reference" | tee -a $O/summary.txt
  done ;;
cpnpmea)
  F2=tests/golden/config/c2_128x256_s11.fa
  for f in $F2 $F3; do
    for m in x 0 x 0; do
      t0=$(date +%s.%N)
      if [ $m = x ]; then unset MLP_MEA_GPU_MIN; else export MLP_MEA_GPU_MIN=$m; fi
      MLP_SRAND_TIME=1700000000 MLP_CLI_TIMES=1 timeout -k 10 120 ./mlprobs_amd/cli/c_p_np_aln -p 1 $f > $O/np$m.out 2> $O/np$m.err || { tail -5 $O/np$m.err; exit 1; }
      t1=$(date +%s.%N)
      echo "$(basename $f) -p 1 MLP_MEA_GPU_MIN=$m wall $(awk "BEGIN{print $t1 - $t0}") $(grep -E '^\[stage\] (refinement|posteriors)|^\[host\]' $O/np$m.err | tr '\n' ' ')" | tee -a $O/summary.txt
    done
    unset MLP_MEA_GPU_MIN
    cmp -s $O/npx.out $O/np0.out && echo "$(basename $f) -p 1 host / device MEA outputs identical" | tee -a $O/summary.txt
  done ;;
chunks)
  # is the wait per allocation size or per process footprint?  each case after
  # a process that held ~150 GB
  P=tools/probe/alloc_chunks
  V=tools/probe/vmm_probe
  for spec in "$P 4 64" "$P 4 64" "$P 64 64" "$P 64 64" "$V 4 64" "$V 4 64" "$P 8 96" "$P 8 96" "$V 8 96" "$V 8 96"; do
    timeout -k 10 200 python3 bench.py --no-cpu --no-e2e --no-qp --relax 0 --no-shards --steps 1 --warmup 0 > /dev/null 2>&1 || exit 1
    t0=$(date +%s.%N)
    timeout -k 10 60 $spec > $O/chunk.txt 2>&1 || { cat $O/chunk.txt; exit 1; }
    t1=$(date +%s.%N)
    echo "== $spec wall $(awk "BEGIN{print $t1 - $t0}") | $(grep -E 'malloc [0-9.]*[1-9][0-9.]* s|create\+map [0-9.]*[1-9]|memset all|reserve' $O/chunk.txt | tr '\n' ';')" | tee -a $O/summary.txt
  done ;;
tottr)
  MLP_TOT_TR=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > $O/tottr_test.log 2>&1 || { tail -20 $O/tottr_test.log; exit 1; }
  echo "MLP_TOT_TR=1 parity + config tests: $(tail -1 $O/tottr_test.log)" | tee -a $O/summary.txt
  for rep in 1 2; do
    for j in 0 1; do
      MLP_TOT_TR=$j timeout -k 10 300 python3 bench.py --no-e2e --no-qp --relax 0 --no-shards --steps 3 --warmup 1 \
        --cpu-pairs 1024 > $O/tr$j.json 2> $O/tr$j.err || { tail -5 $O/tr$j.err; exit 1; }
      python3 -c "
import json; d=json.load(open('$O/tr$j.json'))
k=d['kernels_ms_per_step']; p=d.get('parity') or {}
print('MLP_TOT_TR=$j', 'step %.1f ms' % d['ms_per_step'], ' '.join('%s %.1f' % (a, b) for a, b in k.items()), 'parity max_rel_err', p.get('max_rel_err'))" | tee -a $O/summary.txt
    done
  done ;;
qpprof)
  # kernel statistics of one quickprobs C3 run (construction + refinement:
  # 711 profile posteriors + MEAs on the device)
  export TMPDIR=/tmp
  MLP_CLI_TIMES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/qpprof -o qp -- \
    ./mlprobs_amd/cli/quickprobs $F3 > $O/qpprof.out 2> $O/qpprof.err || { tail -5 $O/qpprof.err; exit 1; }
  grep -E '^\[(stage|host)\]' $O/qpprof.err | tee -a $O/summary.txt
  head -12 $O/qpprof/qp_kernel_stats.csv | cut -d, -f1-4 | tee -a $O/summary.txt ;;
pg)
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > $O/pg_test.log 2>&1 || { tail -20 $O/pg_test.log; exit 1; }
  echo "PF posterior in the Zm slot: parity + config tests: $(tail -1 $O/pg_test.log)" | tee -a $O/summary.txt
  for rep in 1 2; do
    for j in 1 0; do
      MLP_PG_SEPARATE=$j timeout -k 10 300 python3 bench.py --no-e2e --no-qp --relax 0 --no-shards --steps 3 --warmup 1 \
        --cpu-pairs 1024 > $O/pg$j.json 2> $O/pg$j.err || { tail -5 $O/pg$j.err; exit 1; }
      python3 -c "
import json; d=json.load(open('$O/pg$j.json'))
k=d['kernels_ms_per_step']; p=d.get('parity') or {}
print('MLP_PG_SEPARATE=$j', 'step %.1f ms' % d['ms_per_step'], ' '.join('%s %.1f' % (a, b) for a, b in k.items()), 'parity max_rel_err', p.get('max_rel_err'))" | tee -a $O/summary.txt
    done
  done
  for j in 1 0; do
    for rep in 1 2; do
      t0=$(date +%s.%N)
      MLP_PG_SEPARATE=$j MLP_CLI_TIMES=1 timeout -k 10 120 ./mlprobs_amd/cli/c_p_np_aln -p 0 $F3 > $O/pgc.out 2> $O/pgc.err || { tail -5 $O/pgc.err; exit 1; }
      t1=$(date +%s.%N)
      echo "C3 -p 0 MLP_PG_SEPARATE=$j wall $(awk "BEGIN{print $t1 - $t0}") $(grep -E '^\[stage\] posteriors' $O/pgc.err)" | tee -a $O/summary.txt
      cmp -s $O/pgc.out tests/golden/config/c3_512x400_s11.p_0.out && echo "  output = reference" | tee -a $O/summary.txt
    done
  done ;;
meamin)
  # profile MEA cell floor for the device (MLP_MEA_GPU_MIN), both drop-ins
  F2=tests/golden/config/c2_128x256_s11.fa
  for thr in ${THRS:-0 100000 250000 500000 1000000000000}; do
    for spec in "c_p_np_aln -p 0 $F2" "c_p_np_aln -p 1 $F2" "c_p_np_aln -p 0 $F3" "quickprobs $F2" "quickprobs $F3"; do
      set -- $spec
      tag=$(echo "$spec" | tr ' /' '__' | tail -c 40)
      MLP_MEA_GPU_MIN=$thr MLP_SRAND_TIME=1700000000 MLP_CLI_TIMES=1 timeout -k 10 120 ./mlprobs_amd/cli/$spec > $O/mm_$thr$tag.out 2> $O/mm.err || { tail -5 $O/mm.err; exit 1; }
      echo "thr $thr $1 $2 $3 $(basename ${@: -1}): $(grep -E '^\[stage\] (progressive|refinement|construction)' $O/mm.err | tr '\n' ' ')" | tee -a $O/summary.txt
    done
  done
  for spec in "c_p_np_aln -p 0 $F2" "c_p_np_aln -p 1 $F2" "c_p_np_aln -p 0 $F3" "quickprobs $F2" "quickprobs $F3"; do
    tag=$(echo "$spec" | tr ' /' '__' | tail -c 40)
    md5sum $O/mm_*$tag.out | awk '{print $1}' | sort -u | wc -l | xargs echo "distinct outputs over thresholds for $spec:" | tee -a $O/summary.txt
  done ;;
pmc)
  tools/pmc_run.sh gpurun_out/pmc_r03 "--steps 1 --warmup 0 --no-cpu --no-e2e --no-qp --no-shards --relax 1" || exit 1
  echo "pmc passes done" | tee -a $O/summary.txt ;;
qpcli)
  timeout -k 10 600 python3 -u -m pytest tests/test_cli_gpu.py -m gpu -x -q -k quickprobs --timeout 300 --timeout-method thread \
    > $O/qpcli.log 2>&1 || { tail -20 $O/qpcli.log; exit 1; }
  echo "quickprobs CLI tests: $(tail -1 $O/qpcli.log)" | tee -a $O/summary.txt ;;
meatest)
  timeout -k 10 600 python3 -u -m pytest tests/test_cli_gpu.py tests/test_gpu_parity.py -m gpu -x -q -k "quickprobs or profile or cli" \
    --timeout 300 --timeout-method thread > $O/meatest.log 2>&1 || { tail -20 $O/meatest.log; exit 1; }
  echo "CLI + profile tests: $(tail -1 $O/meatest.log)" | tee -a $O/summary.txt ;;
qptimes)
  for rep in 1 2; do
    MLP_PROFILE_TIMES=1 MLP_CLI_TIMES=1 timeout -k 10 120 ./mlprobs_amd/cli/quickprobs $F3 > $O/qpt.out 2> $O/qpt.err || { tail -5 $O/qpt.err; exit 1; }
    grep -E '^\[(stage\] construction|host|profile)' $O/qpt.err | tee -a $O/summary.txt
    [ "$(md5sum < $O/qpt.out | cut -d' ' -f1)" = "1a8db641783cdbef0ee0b16bf46fc611" ] && echo "  output md5 = the earlier runs' (1a8db641783cdbef0ee0b16bf46fc611)" | tee -a $O/summary.txt
  done ;;
post)
  timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > $O/post_test.log 2>&1 || { tail -20 $O/post_test.log; exit 1; }
  echo "parity + config tests: $(tail -1 $O/post_test.log)" | tee -a $O/summary.txt
  for rep in 1 2; do
    timeout -k 10 300 python3 bench.py --no-e2e --no-qp --relax 0 --no-shards --steps 3 --warmup 1 \
      --cpu-pairs 1024 > $O/post.json 2> $O/post.err || { tail -5 $O/post.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/post.json'))
k=d['kernels_ms_per_step']; p=d.get('parity') or {}
print('posterior stage', 'step %.1f ms' % d['ms_per_step'], ' '.join('%s %.1f' % (a, b) for a, b in k.items()), 'parity max_rel_err', p.get('max_rel_err'))" | tee -a $O/summary.txt
  done ;;
teardown)
  F2=tests/golden/config/c2_128x256_s11.fa
  for f in $F2 $F3; do
    for m in 0 1; do
      MLP_CLI_TIMES=1 MLP_PROFILE_TIMES=1 timeout -k 10 120 ./mlprobs_amd/cli/c_p_np_aln -p $m $f > $O/td.out 2> $O/td.err || { tail -5 $O/td.err; exit 1; }
      echo "$(basename $f) -p $m: $(grep -E '^\[(stage\] (refinement|progressive|alignment|context|output)|profile posterior\]|host\])' $O/td.err | tr '\n' ' ')" | tee -a $O/summary.txt
    done
  done ;;
relaxlog)
  MLP_SCRATCH_GB=16 MLP_RELAX_LOG=1 MLP_CLI_TIMES=1 timeout -k 10 120 ./mlprobs_amd/cli/c_p_np_aln -p 0 $F3 > $O/rl.out 2> $O/rl.err || { tail -5 $O/rl.err; exit 1; }
  cat $O/rl.err | tee -a $O/summary.txt ;;
alloc)
  tools/probe/alloc_seq.sh > /dev/null && cat gpurun_out/alloc_seq/summary.txt >> $O/summary.txt ;;
esac
done
cat $O/summary.txt
