#!/bin/bash
# Reference `c_p_np_aln -p 0` outputs on the BASELINE configuration families
# (build container only: oracle/_ref/c_p_np_aln is the reference built from
# /root/reference by `make -C oracle ref`).  C2 (128 sequences) runs on one
# core: its refinement calls the reference's racy parallel BuildPosterior
# (CPNP/MSA.cpp:1562, ProbabilisticModel.h:1223).  C3 (512 sequences) turns
# refinement off (CPNP/MSA.cpp:1502) and the progressive merges use the
# serial weighted BuildPosterior (MSA.cpp:1431), so it may use every core.
set -e
cd "$(dirname "$0")/.."
G=tests/golden/config
python3 -c "
import sys; sys.path.insert(0, '.')
from mlprobs_amd import synth
synth.write_fasta('$G/c2_128x256_s11.fa', synth.family(128, 256, 0.7, seed=11))
synth.write_fasta('$G/c3_512x400_s11.fa', synth.family(512, 400, 0.7, seed=11))
"
taskset -c 0 oracle/_ref/c_p_np_aln -p 0 $G/c2_128x256_s11.fa > $G/c2_128x256_s11.p_0.out
oracle/_ref/c_p_np_aln -p 0 $G/c3_512x400_s11.fa > $G/c3_512x400_s11.p_0.out
# -p 1 (npdoAlign + refinement) on C2 under the tests' fixed clock
# (MLP_SRAND_TIME, read by the reference's time() stand-in oracle/fixtime.c),
# one core (its refinement's BuildPosterior races the same way)
MLP_SRAND_TIME=1700000000 taskset -c 0 oracle/_ref/c_p_np_aln_ft -p 1 $G/c2_128x256_s11.fa > $G/c2_128x256_s11.p_1.out
# the reference QuickProbs CLI on C2 and C3 (its output does not depend on the thread count)
oracle/_ref/quickprobs -t 8 $G/c2_128x256_s11.fa > $G/c2_128x256_s11.qp.out
oracle/_ref/quickprobs -t 8 $G/c3_512x400_s11.fa > $G/c3_512x400_s11.qp.out
