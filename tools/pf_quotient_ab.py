"""A/B of the C_P_NP_Aln partition-function posterior quotient on the sparse
store: the default (zf * Zm) * (1/score * 1/Z) against the
division (zf * Zm) / (score * Z) of the MLP_PF_DIVIDE build, on the C3 family
(pid 0) and the heavy golden families; per family the number of stored entries
present in only one store and of values that differ.  The reference runs the
quotient in x87 long double, so neither form is bit-pinned: both are checked
against it within 1e-4 by the parity tests.

    python tools/pf_quotient_ab.py            (needs lib/libmlpgpu_pfdiv.so: build_variants.py pfdiv=MLP_PF_DIVIDE)
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')

CHILD = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
from mlprobs_amd import synth
from mlprobs_amd.engine import Family
fa, out, pid = sys.argv[2], sys.argv[3], int(sys.argv[4])
seqs = [s for _, s in synth.read_fasta(fa)]
f = Family(seqs)
f.posteriors(pid, 0.132548)
rp, eo, cols, vals = f.export()
d, m, n = f.results()
np.savez(out, rp=rp, eo=eo, cols=cols, vals=vals, dist=d)
f.close()
'''


def store(fa, variant, td, tag, pid):
    out = os.path.join(td, tag + '.npz')
    env = dict(os.environ)
    env.pop('MLP_LIB_VARIANT', None)
    if variant:
        env['MLP_LIB_VARIANT'] = variant
    subprocess.run([sys.executable, '-c', CHILD, ROOT, fa, out, str(pid)], check=True, env=env, timeout=600)
    return np.load(out)


def compare(a, b, lens):
    """Entries per (pair, row, column) present in one store only, and values
    that differ where both have the entry."""
    if np.array_equal(a['rp'], b['rp']) and np.array_equal(a['cols'], b['cols']):
        return {'entries': int(len(a['cols'])), 'one_sided': 0,
                'values_differ': int(np.count_nonzero(a['vals'] != b['vals'])),
                'dist_differ': int(np.count_nonzero(a['dist'] != b['dist']))}
    only, diff, both = 0, 0, 0
    ea, eb = a['eo'], b['eo']
    n = len(lens)
    p = ro = 0
    for x in range(n):
        for y in range(x + 1, n):
            L1 = lens[x]
            ra, rb = a['rp'][ro:ro + L1 + 2], b['rp'][ro:ro + L1 + 2]
            ca, cb = a['cols'][ea[p]:ea[p + 1]], b['cols'][eb[p]:eb[p + 1]]
            va, vb = a['vals'][ea[p]:ea[p + 1]], b['vals'][eb[p]:eb[p + 1]]
            if np.array_equal(ra, rb) and np.array_equal(ca, cb):
                both += len(ca)
                diff += int(np.count_nonzero(va != vb))
            else:
                ka = np.repeat(np.arange(L1 + 1), np.diff(ra[:L1 + 2])).astype(np.int64) * 65536 + ca
                kb = np.repeat(np.arange(L1 + 1), np.diff(rb[:L1 + 2])).astype(np.int64) * 65536 + cb
                common, ia, ib = np.intersect1d(ka, kb, return_indices=True)
                only += len(ka) + len(kb) - 2 * len(common)
                diff += int(np.count_nonzero(va[ia] != vb[ib]))
                both += len(common)
            ro += L1 + 2
            p += 1
    return {'entries': both, 'one_sided': only, 'values_differ': diff,
            'dist_differ': int(np.count_nonzero(a['dist'] != b['dist']))}


def main():
    sys.path.insert(0, ROOT)
    from mlprobs_amd import synth
    fams = []
    with tempfile.TemporaryDirectory() as td:
        c3 = os.path.join(td, 'c3.fa')
        synth.write_fasta(c3, synth.family(512, 400, 0.7, seed=11))
        fams.append(('C3 512x400 s=0.7', c3))
        heavy = os.path.join(ROOT, 'tests', 'golden', 'pipeline_heavy')
        for fn in sorted(os.listdir(heavy)):
            if fn.endswith('.fa'):
                fams.append((fn, os.path.join(heavy, fn)))
        for name, fa in fams:
            a = store(fa, None, td, 'a', 0)
            b = store(fa, 'pfdiv', td, 'b', 0)
            lens = [len(s) for _, s in synth.read_fasta(fa)]
            r = compare(a, b, lens)
            r['family'] = name
            print(json.dumps(r), flush=True)


if __name__ == '__main__':
    main()
