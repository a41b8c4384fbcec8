"""PF posterior vs the oracle on high-magnitude pairs (all-W, repeats)."""
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
cases = []
for L in (30, 50, 70, 90, 110, 130):
    cases.append((f'W{L}', 'W' * L, 'W' * L))
    cases.append((f'W{L}x{L+20}', 'W' * L, 'W' * (L + 20)))
    cases.append((f'C{L}', 'C' * L, 'C' * L))
s0, s4 = fam[0], fam[4]
for k in (130, 140, 150, 158):
    cases.append((f's0[:{k}],s4', s0[:k], s4))
    cases.append((f's0[-{k}:],s4', s0[-k:], s4))
for tag, a, b in cases:
    f = engine.Family([a, b])
    try:
        f.posteriors(3, delta)
    except Exception as e:  # noqa: BLE001
        print(tag, 'error', e, flush=True)
        f.close()
        continue
    rp, cols, vals = f.sparse(0)
    k1, k2 = len(a), len(b)
    post = orc.pair_posterior(m, a, b, 3)
    dense = np.zeros((k1 + 1, k2 + 1), np.float32)
    for i in range(1, k1 + 1):
        dense[i, cols[rp[i]:rp[i + 1]]] = vals[rp[i]:rp[i + 1]]
    ref = post.reshape(k1 + 1, k2 + 1)
    ref = np.where(ref >= 0.01, ref, 0)
    err = np.abs(dense - ref).max()
    print(f'{tag:16s}: max gpu {vals.max() if len(vals) else 0:.6f} ref {ref.max():.6f} max|diff| {err:.2e}',
          flush=True)
    f.close()
