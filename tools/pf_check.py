"""GPU vs oracle posteriors / distances on one family (default: the
near-identical oxx____8t2 real family, pid from the family test)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'oracle'))
import orc  # noqa: E402
from mlprobs_amd import synth, engine  # noqa: E402

path = sys.argv[1] if len(sys.argv) > 1 else 'tests/golden/real/oxx____8t2.fa'
seqs = [s for _, s in synth.read_fasta(path)]
m0 = orc.model(0.132548)
vm, ident, delta = orc.model_adjustment(m0, seqs)
pid = vm % 10
m = orc.model(delta)
fam = engine.Family(seqs)
fam.posteriors(pid, delta)
D = fam.distances()
n = len(seqs)
k = 0
worst = 0
for a in range(n):
    for b in range(a + 1, n):
        post = orc.pair_posterior(m, seqs[a], seqs[b], pid)
        sc = orc.mea(len(seqs[a]), len(seqs[b]), post)
        d = np.float32(1) - np.float32(sc) / np.float32(min(len(seqs[a]), len(seqs[b])))
        rp, cols, vals = fam.sparse(k)
        if D[a, b] < 0.001 or abs(D[a, b] - d) > 1e-4:
            dense = post.reshape(len(seqs[a]) + 1, len(seqs[b]) + 1)
            gv = vals.max() if len(vals) else 0
            print(f'pair {a},{b} L {len(seqs[a])},{len(seqs[b])} dist gpu {D[a, b]:.7f} oracle {d:.7f} '
                  f'max post gpu {gv:.7f} oracle {dense.max():.7f}', flush=True)
        k += 1
print('pid', pid, 'delta', delta)
