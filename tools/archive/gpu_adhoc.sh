#!/bin/bash
# which c5 process is slow on the box: the drop-in's host path or the reference CLI?
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/c5probe
mkdir -p $O
python3 - <<'PY'
import json, lzma, os
fams = json.load(lzma.open('tests/golden/sweep.json.xz', 'rt'))
names = [k for k in sorted(fams) if k.split('/')[0] in ('ox', 'sabre') and 'p_0' in fams[k]][::15]
open('/tmp/c5_0.fa', 'wb').write(fams[names[0]]['fa'].encode('latin-1'))
print(names[0], fams[names[0]]['n'], fams[names[0]]['cells'])
PY
nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; taskset -p $$
t() { local t0=$(date +%s.%N); timeout -k 5 $1 "${@:2}" > /dev/null 2>&1; local rc=$?; echo "rc=$rc $(awk "BEGIN{print $(date +%s.%N) - $t0}") s: ${@:2}"; }
t 60 env MLP_CLI_TIMES=1 ./mlprobs_amd/cli/c_p_np_aln -G /tmp/c5_0.fa
t 60 ./mlprobs_amd/cli/c_p_np_aln -p 0 /tmp/c5_0.fa
t 60 env MLP_HOST_THREADS=1 ./mlprobs_amd/cli/c_p_np_aln -p 0 /tmp/c5_0.fa
t 30 env OMP_NUM_THREADS=1 ./oracle/_ref/c_p_np_aln -p 0 /tmp/c5_0.fa
t 30 env OMP_NUM_THREADS=4 ./oracle/_ref/c_p_np_aln -p 0 /tmp/c5_0.fa
t 30 env OMP_NUM_THREADS=16 ./oracle/_ref/c_p_np_aln -p 0 /tmp/c5_0.fa
t 30 env OMP_NUM_THREADS=16 OMP_WAIT_POLICY=passive ./oracle/_ref/c_p_np_aln -p 0 /tmp/c5_0.fa
