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
