"""Sweep truncations of the failing pair (s0, s4) of oxx____8t2 at pid 3."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'oracle'))
import orc  # noqa: E402
from mlprobs_amd import synth, engine  # noqa: E402

fam = [s for _, s in synth.read_fasta('tests/golden/real/oxx____8t2.fa')]
delta = 0.16785800457000732
m = orc.model(delta)
s0, s4 = fam[0], fam[4]
for k1 in (40, 80, 120, 158):
    for k2 in (60, 100, 140, 171):
        a, b = s0[:k1], s4[:k2]
        f = engine.Family([a, b])
        f.posteriors(3, delta)
        rp, cols, vals = f.sparse(0)
        post = orc.pair_posterior(m, a, b, 3)
        dense = np.zeros((k1 + 1, k2 + 1), np.float32)
        for i in range(1, k1 + 1):
            dense[i, cols[rp[i]:rp[i + 1]]] = vals[rp[i]:rp[i + 1]]
        ref = post.reshape(k1 + 1, k2 + 1)
        ref = np.where(ref >= 0.01, ref, 0)
        err = np.abs(dense - ref).max()
        print(f'k1 {k1} k2 {k2}: max gpu {vals.max() if len(vals) else 0:.6f} ref {ref.max():.6f} '
              f'max|diff| {err:.2e}', flush=True)
        f.close()
