"""Helpers to load the committed reference fixtures (tests/golden/)."""
import glob
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def manifest():
    with open(os.path.join(GOLDEN, 'manifest.json')) as fh:
        return json.load(fh)


def pair_names():
    return sorted(os.path.basename(p)[5:-4] for p in glob.glob(os.path.join(GOLDEN, 'pair_*.npz')))


def family_names():
    return sorted(os.path.basename(p)[7:-4] for p in glob.glob(os.path.join(GOLDEN, 'family_*.npz')))


def load_pair(name):
    d = dict(np.load(os.path.join(GOLDEN, f'pair_{name}.npz')))
    d['s1'] = bytes(d['s1']).decode()
    d['s2'] = bytes(d['s2']).decode()
    return d


def load_family(name):
    d = dict(np.load(os.path.join(GOLDEN, f'family_{name}.npz')))
    d['seqs'] = [str(s) for s in d['seqs']]
    for k in ('variance_mean', 'delta', 'pid', 'reps'):
        d[k] = np.asarray(d[k]).reshape(-1)[0]
    return d


def family_csrs(d, it):
    """Split a family's iteration-`it` CSR into per-pair (rowptr, cols, vals)."""
    lens = d['lens']
    n = len(lens)
    rp_all, c_all, v_all = d[f'it{it}.rowptr'], d[f'it{it}.cols'], d[f'it{it}.vals']
    res, r, e = [], 0, 0
    for a in range(n):
        for b in range(a + 1, n):
            rp = rp_all[r:r + lens[a] + 2]
            nnz = int(rp[-1])
            res.append((rp.astype(np.int32), c_all[e:e + nnz].astype(np.int32), v_all[e:e + nnz].astype(np.float32)))
            r += lens[a] + 2
            e += nnz
    return res


def pairs_of(n):
    return [(a, b) for a in range(n) for b in range(a + 1, n)]


def qp_pair_names():
    return sorted(os.path.basename(p)[8:-4] for p in glob.glob(os.path.join(GOLDEN, 'qp_pair_*.npz')))


def load_qp_pair(name):
    """QuickProbs posterior-stage vectors (tests/golden/gen_golden.py gen_qp)."""
    d = dict(np.load(os.path.join(GOLDEN, f'qp_pair_{name}.npz')))
    d['s1'] = bytes(d['s1']).decode()
    d['s2'] = bytes(d['s2']).decode()
    return d


def qp_family_names():
    return sorted(os.path.basename(p)[10:-4] for p in glob.glob(os.path.join(GOLDEN, 'qp_family_*.npz')))


def load_qp_family(name):
    d = dict(np.load(os.path.join(GOLDEN, f'qp_family_{name}.npz')))
    d['seqs'] = [str(s) for s in d['seqs']]
    d['iters'] = int(np.asarray(d['iters']).reshape(-1)[0])
    return d


def qp_family_csrs(d, it):
    """Per-pair (rowptr, cols, q / 65535) of round `it` (0 = posterior stage)."""
    lens = [len(s) for s in d['seqs']]
    n = len(lens)
    rp, eo = d[f'it{it}.row_ptr'], d[f'it{it}.ent_off']
    cols, q = d[f'it{it}.cols'], d[f'it{it}.qvals']
    out, ro, p = [], 0, 0
    for a in range(n):
        for b in range(a + 1, n):
            r = rp[ro:ro + lens[a] + 2].astype(np.int32)
            ro += lens[a] + 2
            out.append((r, cols[eo[p]:eo[p + 1]].astype(np.int32),
                        q[eo[p]:eo[p + 1]].astype(np.float32) / np.float32(65535)))
            p += 1
    return out
