"""Sparsity statistics of the relaxation inputs (design data for relax.hip).

Runs the C3 posterior stage on the GPU, exports the sparse set and prints
row-length / row-span histograms plus per-task staging sizes for a sample
of (x, y, z, 64-row chunk) relaxation tasks.  Run on the GPU box:
    python tools/relax_stats.py [N L]
"""
import sys
import os
import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
from mlprobs_amd import synth, engine  # noqa: E402


def block(fam, csr, a, b):
    """(row_ptr, cols, vals) of P(a, b) for any a != b (transposed if a > b)."""
    rp, eo, cols, vals = csr
    if a < b:
        p = engine.pair_index(fam.n, a, b)
        r = rp[fam.rp_off[p]:fam.rp_off[p + 1]].astype(np.int64)
        return r, cols[eo[p]:eo[p + 1]].astype(np.int64), vals[eo[p]:eo[p + 1]]
    r, c, v = block(fam, csr, b, a)
    La, Lb = fam.lens[b], fam.lens[a]
    rows = np.repeat(np.arange(La + 2), np.diff(r, append=r[-1])[:La + 2])[:len(c)]
    order = np.lexsort((rows, c))
    tc, tv = c[order], rows[order]
    trp = np.zeros(Lb + 2, np.int64)
    np.add.at(trp, tc + 1, 1)
    trp = np.cumsum(trp)
    return trp, tv, v[order]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 400
    seqs = [s for _, s in synth.family(n, L, 0.7, seed=11)]
    fam = engine.Family(seqs)
    fam.posteriors(0, 0.0)
    csr = fam.export()
    rp, eo, cols, vals = csr
    for it in range(2):
        rp, eo, cols, vals = csr
        lens_all = []
        spans = []
        for p in range(0, fam.npairs, max(1, fam.npairs // 4000)):
            r = rp[fam.rp_off[p]:fam.rp_off[p + 1]].astype(np.int64)
            c = cols[eo[p]:eo[p + 1]].astype(np.int64)
            rl = np.diff(r)[1:]
            lens_all.append(rl)
            ne = rl > 0
            s = r[1:-1][ne]
            e = r[2:][ne] - 1
            spans.append(c[e] - c[s] + 1)
        rl = np.concatenate(lens_all)
        sp = np.concatenate(spans)
        print(f'iteration {it}: total nnz {len(cols)} ({len(cols) / fam.npairs / L:.2f}/row)')
        print('  row nnz pct 50/90/99/max', np.percentile(rl, [50, 90, 99]), rl.max())
        print('  row span pct 50/90/99/99.9/max', np.percentile(sp, [50, 90, 99, 99.9]), sp.max(),
              'frac>32', (sp > 32).mean(), 'frac>64', (sp > 64).mean())
        rng = np.random.default_rng(1)
        segA, bandR, bandE, visits, vmax = [], [], [], [], []
        for _ in range(300):
            x, y, z = rng.choice(n, 3, replace=False)
            if x > y:
                x, y = y, x
            Ar, Ac, _ = block(fam, csr, x, z)
            Br, Bc, _ = block(fam, csr, z, y)
            for i0 in range(1, fam.lens[x] + 1, 64):
                i1 = min(i0 + 64, fam.lens[x] + 1)
                a0, a1 = Ar[i0], Ar[i1]
                segA.append(a1 - a0)
                if a1 == a0:
                    continue
                ks = Ac[a0:a1]
                k0, k1 = ks.min(), ks.max()
                bandR.append(k1 - k0 + 1)
                bandE.append(Br[k1 + 1] - Br[k0])
                bl = np.diff(Br)[ks]
                rows = np.repeat(np.arange(i0, i1), np.diff(Ar[i0:i1 + 1]))
                per = np.bincount(rows - i0, weights=bl, minlength=64)
                visits.append(per.sum())
                vmax.append(per.max())
        f = lambda a: np.percentile(a, [50, 90, 99]).round(1).tolist() + [int(np.max(a))]
        print('  A seg entries/chunk 50/90/99/max', f(segA))
        print('  B band rows 50/90/99/max', f(bandR), ' entries', f(bandE))
        print('  visits/chunk', f(visits), ' max-lane visits', f(vmax),
              ' util', np.sum(visits) / 64 / np.sum(vmax))
        if it == 0:
            fam.relax(1)
            csr = fam.export()


if __name__ == '__main__':
    main()
