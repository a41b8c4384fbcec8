# (experiment of round 6: not kept)
#!/bin/bash
# wall time of c_p_np_aln -p 0 on C2, normal exit vs _exit after the output, alternating
export TMPDIR=/tmp
F=tests/golden/config/c2_128x256_s11.fa
for i in 1 2 3 4 5; do
  for mode in normal quick; do
    if [ $mode = quick ]; then export MLP_EXP_QUICK_EXIT=1; else unset MLP_EXP_QUICK_EXIT; fi
    s=$(date +%s.%N)
    MLP_CLI_TIMES=1 timeout -k 5 60 ./mlprobs_amd/cli/c_p_np_aln -p 0 $F > /tmp/o_$mode.txt 2> /tmp/e_$mode.txt
    e=$(date +%s.%N)
    init=$(grep "device init" /tmp/e_$mode.txt | awk '{print $4}')
    echo "$mode $(awk "BEGIN{print $e - $s}") init $init $(cmp -s /tmp/o_$mode.txt tests/golden/config/c2_128x256_s11.p_0.out && echo same || echo DIFF)"
  done
done
