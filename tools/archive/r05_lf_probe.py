"""r05 diagnosis: the deferred batch finish with the lane fold at a 1 GB scratch -- which outputs differ
(per family: store arrays and results compared with the finish-first run; one child process per setting)."""
import os
import subprocess
import sys

import numpy as np

FAMS = ((48, 300, 0.7, 31, 0), (40, 260, 0.35, 32, 0), (6, 900, 0.6, 34, 0))
NAMES = ['rowptr', 'ent_off', 'cols', 'vals', 'dist', 'mea', 'nnz']

if len(sys.argv) > 1:   # child: dump every family's arrays
    sys.path.insert(0, os.getcwd())
    from mlprobs_amd import synth
    from mlprobs_amd.engine import Family
    d = {}
    for k, (n, L, s, seed, pid) in enumerate(FAMS):
        seqs = [q for _, q in synth.family(n, L, s, seed=seed)]
        f = Family(seqs)
        f.set_scratch(1 << 30)
        f.posteriors(pid, 0.132548)
        for j, a in enumerate(list(f.export()) + list(f.results())):
            d[f'f{k}_{j}'] = np.asarray(a)
        f.close()
    np.savez(sys.argv[1], **d)
    sys.exit(0)

res = {}
for v in ('0', '1'):
    out = f'/tmp/lfp_{v}.npz'
    subprocess.run([sys.executable, __file__, out], check=True, env=dict(os.environ, MLP_TEST_DEFER_FINISH=v, MLP_TEST_TOT_LANEFOLD='1'))
    res[v] = np.load(out)
for k in range(len(FAMS)):
    row = []
    for j in range(7):
        x, y = res['0'][f'f{k}_{j}'], res['1'][f'f{k}_{j}']
        row.append('same' if np.array_equal(x, y) else (f'DIFF {int((x != y).sum())}/{x.size}' if x.shape == y.shape else f'SHAPE {x.shape} {y.shape}'))
    print('family', k, row, flush=True)
    x, y = res['0'][f'f{k}_4'], res['1'][f'f{k}_4']
    if x.shape == y.shape and not np.array_equal(x, y):
        idx = np.nonzero(x != y)
        print('   dist first diffs at', [tuple(int(t) for t in z) for z in list(zip(*idx))[:8]])
