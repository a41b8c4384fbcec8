"""Wave-exact simulation of k_relax_tile's word walk and hit loops on a C3-like
family (no GPU): for each output pair (x, y) and each z, every mask cell's
overlap of the A_z row-i and C_z row-j span bitmaps is walked two 32-column
words per trip, the hit loops run per word; a wave's slot runs its 64 cells
in lockstep, so it issues max-over-lanes trips.  Reports the lane efficiency
of the word walk and the hit loops for several cell orders (the kernel uses
CSR order), and the trips a single 64-bit hit loop per word pair or a flat
hit loop per cell would issue.

    python tools/relax_divergence_sim.py [n] [outputs]     (default 40 12)
"""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path.insert(0, ROOT)
from mlprobs_amd import synth  # noqa: E402
from mlprobs_amd.engine import Family  # noqa: E402

POP = np.array([bin(i).count('1') for i in range(1 << 16)], np.uint8)
W = 16


def popc(x):
    return POP[x & 0xffff] + POP[x >> 16]


def store(n):
    seqs = [s for _, s in synth.family(n, 400, 0.7, seed=11)]  # the bench family's first n sequences
    f = Family(seqs, host=True)
    f.posteriors(0, 0.132548)
    rp, eo, cols, vals = f.export()
    return rp, eo, cols, f.lens, f.rp_off


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    nout = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    rp, eo, cols, lens, rp_off = store(n)
    pidx = lambda a, b: a * n - a * (a + 1) // 2 + (b - a - 1)
    cache = {}

    def image(a, b):  # rows of P(a, b): (first word, words spanned, bitmap words)
        if (a, b) in cache:
            return cache[(a, b)]
        if a < b:
            p = pidx(a, b)
            r = rp[rp_off[p]:rp_off[p] + lens[a] + 2]
            c = cols[eo[p]:eo[p + 1]].astype(np.int64)
            rows = np.repeat(np.arange(lens[a] + 1), np.diff(r[:lens[a] + 2]))
        else:
            p = pidx(b, a)
            r = rp[rp_off[p]:rp_off[p] + lens[b] + 2]
            rows = cols[eo[p]:eo[p + 1]].astype(np.int64)
            c = np.repeat(np.arange(lens[b] + 1), np.diff(r[:lens[b] + 2]))
        R = lens[a] + 1
        dense = np.zeros((R + 1, (max(lens) + 2 + 31) // 32 * 32 + 64), bool)
        dense[rows, c] = True
        words = np.packbits(dense.reshape(R + 1, -1, 32)[:, :, ::-1], axis=2, bitorder='big').view('>u4')[:, :, 0]
        words = words.astype(np.uint32)
        nz = words != 0
        anyw = nz.any(1)
        first = np.where(anyw, nz.argmax(1), 0)
        last = np.where(anyw, nz.shape[1] - 1 - nz[:, ::-1].argmax(1), -1)
        cache[(a, b)] = (first, np.where(anyw, last - first + 1, 0), words)
        return cache[(a, b)]

    orders = ['csr', 'row-width', 'column-major', 'total-hits', 'random']
    acc = {o: np.zeros(5) for o in orders}
    extra = {'pair64': 0, 'flat': 0}
    outs = [(x, y) for x in range(n) for y in range(x + 1, n)]
    for k in np.random.default_rng(1).permutation(len(outs))[:nout]:
        x, y = outs[k]
        p = pidx(x, y)
        r = rp[rp_off[p]:rp_off[p] + lens[x] + 2]
        ci = np.repeat(np.arange(lens[x] + 1), np.diff(r[:lens[x] + 2]))
        cj = cols[eo[p]:eo[p + 1]].astype(np.int64)
        N = len(ci)
        per_z = []
        for z in range(n):
            if z in (x, y):
                continue
            fa, na, wa = image(x, z)
            fc, nc, wc = image(y, z)
            a0, c0 = fa[ci], fc[cj]
            ws, we = np.maximum(a0, c0), np.minimum(a0 + na[ci], c0 + nc[cj])
            trips = np.maximum(0, (we - ws + 1) // 2)
            trips[(na[ci] == 0) | (nc[cj] == 0)] = 0
            h = np.zeros((N, 2 * W), np.int64)
            for q in range(2 * W):
                ok = ws + q < we
                if not ok.any():
                    break
                wi = np.minimum(ws + q, wa.shape[1] - 1)
                h[:, q] = np.where(ok, popc(wa[ci, wi] & wc[cj, wi]), 0)
            per_z.append((trips, h))
        tot_hits = sum(h.sum(1) for _, h in per_z)
        width = np.diff(r[:lens[x] + 2])[ci]
        perms = {'csr': np.arange(N), 'row-width': np.argsort(-width, kind='stable'),
                 'column-major': np.lexsort((ci, cj)), 'total-hits': np.argsort(-tot_hits, kind='stable'),
                 'random': np.random.default_rng(0).permutation(N)}
        G = (N + 63) // 64
        for o in orders:
            perm = perms[o]
            for trips, h in per_z:
                t = np.zeros(G * 64, np.int64)
                t[:N] = trips[perm]
                hh = np.zeros((G * 64, 2 * W), np.int64)
                hh[:N] = h[perm]
                t, hh = t.reshape(G, 64), hh.reshape(G, 64, 2 * W)
                acc[o] += (t.max(1).sum(), hh.max(1).sum(), t.sum(), hh.sum(), G)
                if o == 'csr':
                    extra['pair64'] += hh.reshape(G, 64, W, 2).sum(3).max(1).sum()
                    extra['flat'] += hh.sum(2).max(1).sum()
    for o in orders:
        wt, wh, lt, lh, gz = acc[o]
        print('%-12s lane efficiency: word walk %.3f, hit loops %.3f | per wave-slot and z: %.2f trips, %.2f hit trips'
              % (o, lt / 64 / wt, lh / 64 / wh, wt / gz, wh / gz))
    print('csr: hit trips %d as two loops per word pair, %d as one 64-bit loop per pair, %d as one loop per cell'
          % (acc['csr'][1], extra['pair64'], extra['flat']))


if __name__ == '__main__':
    main()
