"""Checker-side forest evaluator (numpy) for the pipeline tests and the
fixture generator: reads mlprobs_amd/classifier/*.forest (written by
tools/export_forests.py) and predicts one sample the way scikit-learn 0.21.3's
RandomForestClassifier.predict does (features as float32, x <= threshold
goes left, per-tree class weights normalised, summed in tree order, divided
by the tree count, first maximum).  The product evaluator is C++
(mlprobs_amd/cli/pipeline.cpp, Forest); this one exists to check it and to
cross-check both against scikit-learn's own predict (tests/test_pipeline.py)."""
import os
import struct

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODELS = os.path.join(ROOT, 'mlprobs_amd', 'classifier')


def load_forest(name):
    with open(os.path.join(MODELS, f'{name}.forest'), 'rb') as fh:
        buf = fh.read()
    assert buf[:4] == b'MLPF'
    ver, nt, nf, nc = struct.unpack_from('<4I', buf, 4)
    assert ver == 1
    pos = 20
    classes = np.frombuffer(buf, '<f8', nc, pos)
    pos += 8 * nc
    trees = []
    for _ in range(nt):
        (n,) = struct.unpack_from('<I', buf, pos)
        pos += 4
        arrs = []
        for dt, cnt in (('<i4', n), ('<i4', n), ('<i4', n), ('<f8', n), ('<f8', n * nc)):
            a = np.frombuffer(buf, dt, cnt, pos)
            pos += a.nbytes
            arrs.append(a)
        arrs[4] = arrs[4].reshape(n, nc)
        trees.append(tuple(arrs))
    assert pos == len(buf)
    return {'classes': classes, 'n_features': nf, 'trees': trees}


def load_para(name):
    with open(os.path.join(MODELS, f'{name}.para')) as fh:
        return [float(x) for x in fh.read().splitlines()]


def predict_proba(forest, x):
    xf = np.asarray(x, np.float64).astype(np.float32)
    allp = np.zeros(len(forest['classes']), np.float64)
    for left, right, feat, thr, val in forest['trees']:
        node = 0
        while left[node] != -1:
            node = left[node] if float(xf[feat[node]]) <= thr[node] else right[node]
        p = val[node].copy()
        norm = p.sum()
        if norm == 0.0:
            norm = 1.0
        allp += p / norm
    return allp / len(forest['trees'])


def predict(forest, x):
    return float(forest['classes'][int(np.argmax(predict_proba(forest, x)))])


def normalise(raw, para):
    return [(float(raw[i]) - para[i * 2 + 1]) / (para[i * 2] - para[i * 2 + 1]) for i in range(len(raw))]
