"""Isolate the PF posterior error on near-identical pairs: 2-sequence
families at pid 3 (PF only) against the oracle."""
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
rng = np.random.default_rng(5)
A = 'ARNDCQEGHILKMFPSTWYV'
cases = [('s0,s4', fam[0], fam[4]), ('s4,s0', fam[4], fam[0]), ('s4,s5', fam[4], fam[5]),
         ('s0,s0', fam[0], fam[0]), ('s4,s4', fam[4], fam[4])]
for L in (60, 100, 150, 200, 300):
    s = ''.join(rng.choice(list(A), L))
    cases.append((f'ident{L}', s, s))
    cases.append((f'ident{L}-trunc', s, s[: L - 13]))
for tag, a, b in cases:
    f = engine.Family([a, b])
    f.posteriors(3, delta)
    rp, cols, vals = f.sparse(0)
    d = f.distances()[0, 1]
    post = orc.pair_posterior(m, a, b, 3)
    sc = orc.mea(len(a), len(b), post)
    dref = np.float32(1) - np.float32(sc) / np.float32(min(len(a), len(b)))
    print(f'{tag:14s} L {len(a)},{len(b)} dist gpu {d:.6f} ref {dref:.6f} max gpu {vals.max():.6f} '
          f'ref {post.max():.6f}', flush=True)
    f.close()
