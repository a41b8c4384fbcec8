"""Device MEA (mlp_profile_mea) timing against the profile sizes: a small
QuickProbs family, its profile posterior left on the device at L1 x L2
columns (the profiles' sequences gapped to those widths), then K MEA calls
timed on the host clock (kernel + its copies and traceback).

    python tools/mea_bench.py [K]      (run under rocprofv3 --kernel-trace
                                        --stats for the kernel's own time)
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
from mlprobs_amd import synth  # noqa: E402
from mlprobs_amd.engine import Family, PID_QP  # noqa: E402




def gapped(rng, s, L):
    pos = np.sort(rng.choice(np.arange(1, L + 1), size=len(s), replace=False))
    return np.concatenate([[0], pos]).astype(np.int32)


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    rng = np.random.default_rng(5)
    seqs = [x for _, x in synth.family(6, 40, 0.6, seed=5)]
    fam = Family(seqs)
    fam.posteriors(PID_QP, 0.0)
    w = rng.uniform(0.1, 0.3, len(seqs)).astype(np.float32)
    fam.relax_qp(1, w)
    A, B = [0, 1, 2], [3, 4, 5]
    for L1, L2 in [(60, 600), (60, 2000), (500, 500), (1000, 1000), (1000, 3000)]:
        mA = [gapped(rng, seqs[k], L1) for k in A]
        mB = [gapped(rng, seqs[k], L2) for k in B]
        fam.profile_defer(True)
        fam.profile_posterior(w, A, mA, L1, B, mB, L2)
        fam.profile_mea(L1, L2)
        t0 = time.perf_counter()
        for _ in range(K):
            fam.profile_mea(L1, L2)
        dt = (time.perf_counter() - t0) / K
        fam.profile_defer(False)
        print(f'L1 {L1} L2 {L2}: {dt * 1e3:.3f} ms per MEA call', flush=True)
    fam.close()


if __name__ == '__main__':
    main()
