"""How many posterior floats of the GPU partition-function path differ from
the oracle (x87 long double, bit-exact with the reference), and by how many
ulps.  Usage (GPU box): python tools/pf_exactness.py FASTA PID"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
import orc  # noqa: E402
from mlprobs_amd import synth  # noqa: E402
from mlprobs_amd.engine import Family  # noqa: E402


def main():
    seqs = [s for _, s in synth.read_fasta(sys.argv[1])]
    pid = int(sys.argv[2])
    delta = float(sys.argv[3]) if len(sys.argv) > 3 else 0.132548
    m = orc.model(delta)
    fam = Family(seqs)
    fam.posteriors(pid, delta)
    n = len(seqs)
    k = 0
    tot = diff = struct = 0
    maxulp = 0
    for a in range(n):
        for b in range(a + 1, n):
            post = orc.pair_posterior(m, seqs[a], seqs[b], pid)
            rp, cols, vals = orc.sparsify(len(seqs[a]), len(seqs[b]), post)
            r2, c2, v2 = fam.sparse(k)
            if not (np.array_equal(rp, r2) and np.array_equal(cols, c2)):
                struct += 1
            else:
                d = vals.view(np.int32).astype(np.int64) - v2.view(np.int32).astype(np.int64)
                diff += int(np.count_nonzero(d))
                maxulp = max(maxulp, int(np.abs(d).max()) if len(d) else 0)
            tot += len(vals)
            k += 1
    print(f'pid {pid}: {tot} entries, {diff} differ (max {maxulp} ulp), {struct} pairs with a different pattern')


if __name__ == '__main__':
    main()
