"""The drop-in's host path (mlp_ctx_create_host, mlprobs_amd/csrc/
host_backend.cpp): c_p_np_aln runs families up to MLP_HOST_MAX_CELLS
(4e6 pair-cells) on the host CPU without initialising the GPU runtime, so
these tests run the real CLI binary in the CPU suite:

* every golden family of the reference CLI under the threshold (tests/golden
  cli, real, edge, np), all modes (-G, -p 0, -p 0 -c 0 -ir 0, -p 1 -ir 0,
  -p 1 under the golden run's fixed clock): byte-identical;
* the parity sweep's c_p_np_aln runs (tests/golden/sweep.json.xz, 878
  families of the reference's TEST sets, -G and -p 0): byte-identical;
* the host context through the C ABI against the oracle: posteriors of every
  pid and of npdoAlign's pair body, relaxation, the family test.
"""
import json
import lzma
import os
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import orc
from goldens import GOLDEN
from mlprobs_amd import synth
from mlprobs_amd.engine import Family

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, 'mlprobs_amd', 'cli', 'c_p_np_aln')
HOST_MAX = 4e6
NP_TIME = '1700000000'


def _cells(fa):
    L = [len(s) for _, s in synth.read_fasta(fa)]
    return sum((L[a] + 1) * (L[b] + 1) for a in range(len(L)) for b in range(a + 1, len(L)))


def _runs():
    """(family, fasta, args, golden output path) of every golden CLI output."""
    out = []
    for name in ('bb11028', 'div12', 'sim8'):
        fa = os.path.join(GOLDEN, 'cli', f'{name}.fa')
        out += [(name, fa, ['-G'], os.path.join(GOLDEN, 'cli', f'{name}_G.out')),
                (name, fa, ['-p', '0'], os.path.join(GOLDEN, 'cli', f'{name}_p_0.out')),
                (name, fa, ['-p', '0', '-c', '0', '-ir', '0'], os.path.join(GOLDEN, 'cli', f'{name}_p_0_c_0_ir_0.out'))]
    for sub in ('real', 'edge'):
        d = os.path.join(GOLDEN, sub)
        for f in sorted(os.listdir(d)):
            if not f.endswith('.fa'):
                continue
            name = f[:-3]
            for tag, args in (('G', ['-G']), ('p_0', ['-p', '0'])):
                g = os.path.join(d, f'{name}.{tag}.out')
                if os.path.exists(g):
                    out.append((name, os.path.join(d, f), args, g))
    npd = os.path.join(GOLDEN, 'np')
    for f in sorted(os.listdir(npd)):
        if f.endswith('.p_1.out'):
            name = f[:-len('.p_1.out')]
            fa = next(os.path.join(GOLDEN, s, f'{name}.fa') for s in ('cli', 'real', 'edge')
                      if os.path.exists(os.path.join(GOLDEN, s, f'{name}.fa')))
            out += [(name, fa, ['-p', '1', '-ir', '0'], os.path.join(npd, f'{name}.p_1_ir_0.out')),
                    (name, fa, ['-p', '1'], os.path.join(npd, f'{name}.p_1.out'))]
    return out


def test_cli_goldens_on_host_path():
    runs = [r for r in _runs() if _cells(r[1]) <= HOST_MAX]
    assert len(runs) >= 150

    def one(r):
        name, fa, args, gold = r
        p = subprocess.run([BIN, *args, fa], capture_output=True, timeout=300,
                           env=dict(os.environ, MLP_SRAND_TIME=NP_TIME, MLP_HOST_THREADS='2'))
        with open(gold, 'rb') as fh:
            return name, args, p.returncode == 0 and p.stderr == b'' and p.stdout == fh.read()

    with ThreadPoolExecutor(4) as ex:
        bad = [(n, a) for n, a, ok in ex.map(one, runs) if not ok]
    assert not bad, bad


def test_parity_sweep_on_host_path(tmp_path):
    """tools/parity_sweep.py's c_p_np_aln half (-G and -p 0 on 878 families)."""
    out = tmp_path / 'sweep.txt'
    subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'parity_sweep.py'), str(out), '8', 'G,p_0'],
                   check=True, capture_output=True, timeout=1200)
    text = out.read_text()
    assert 'G: 878/878 byte-identical' in text and 'p_0: 878/878 byte-identical' in text, text
    assert 'MISMATCH' not in text


@pytest.mark.parametrize('pid', [0, 2, 3, 32, 34, 35])
def test_host_context_vs_oracle(pid):
    """mlp_posteriors on the host context: bit-exact to the oracle (the PF in
    long double like the reference), then one relaxation round."""
    seqs = [s for _, s in synth.family(7, 90, 0.6, seed=20 + pid)]
    delta = 0.132548
    fam = Family(seqs, host=True)
    fam.posteriors(pid, delta)
    n = len(seqs)
    pairs = np.arange(n * (n - 1) // 2)
    dist, mea, rp, eo, cols, vals = orc.pairs_csr(orc.model(delta), seqs, pid, pairs)
    g_rp, g_eo, g_cols, g_vals = fam.export()
    gd, gm, _ = fam.results()
    np.testing.assert_array_equal(g_rp, rp)
    np.testing.assert_array_equal(g_eo, eo)
    np.testing.assert_array_equal(g_cols.astype(np.int32), cols)
    np.testing.assert_array_equal(g_vals, vals)
    np.testing.assert_array_equal(gd, dist)
    if not pid & orc.NPDO:
        np.testing.assert_array_equal(gm, mea)
    lens = [len(s) for s in seqs]
    ref1 = orc.relax(lens, [(r.astype(np.int32), c.astype(np.int32), v) for r, c, v in
                            (fam.sparse(k) for k in range(len(pairs)))])
    fam.relax(1)
    for k in range(len(pairs)):
        r, c, v = fam.sparse(k)
        np.testing.assert_array_equal(r, ref1[k][0])
        np.testing.assert_array_equal(c.astype(np.int32), ref1[k][1])
        np.testing.assert_array_equal(v, ref1[k][2])
    fam.close()


def test_host_context_family_test():
    """ModelAdjustmentTest on the host context against the oracle's."""
    seqs = [s for _, s in synth.family(9, 110, 0.5, seed=41)]
    fam = Family(seqs, host=True)
    ident, _, delta, code = fam.model_adjustment()
    vm, o_ident, o_delta = orc.model_adjustment(orc.model(0.132548), seqs)
    assert code == vm and np.float32(ident) == np.float32(o_ident) and np.float32(delta) == np.float32(o_delta)
    fam.close()


# ---- QuickProbs on the host context (quickprobs drop-in, small families)
QP_BIN = os.path.join(ROOT, 'mlprobs_amd', 'cli', 'quickprobs')


def _qp_expected(seqs, a, b):
    h, g, p, dist = orc.qp_pair(orc.model(-1.0), seqs[a], seqs[b])
    rp, cols, q = orc.qp_sparsify(len(seqs[a]), len(seqs[b]), p)
    return (rp, cols, q.astype(np.float32) / np.float32(65535)), dist


@pytest.mark.parametrize('n,L,s,iters,seed,sel', [(9, 140, 0.6, 2, 71, False), (12, 90, 0.7, 3, 73, False),
                                                  (14, 120, 0.6, 2, 74, True), (6, 60, 0.2, 1, 76, True)])
def test_host_context_qp_stage_vs_oracle(n, L, s, iters, seed, sel):
    """QuickProbs' posterior stage and selective consistency rounds on the host
    context: bit-exact to the oracle's restatement (the GPU twin of this test
    is test_gpu_parity.py::test_qp_stage_vs_oracle)."""
    from mlprobs_amd.engine import PID_QP
    seqs = [x for _, x in synth.family(n, L, s, seed=seed)]
    rng = np.random.default_rng(seed)
    w = rng.uniform(1, 30, n).astype(np.float32)
    seld = None
    if sel:
        seld = rng.integers(2, n + 1, (n, n)).astype(np.float32)
        seld = np.minimum(seld, seld.T)
        np.fill_diagonal(seld, 0)
    fam = Family(seqs, host=True)
    fam.posteriors(PID_QP, 0.0)
    D = fam.distances()
    cur, k = [], 0
    for a in range(n):
        for b in range(a + 1, n):
            ref, dist = _qp_expected(seqs, a, b)
            r, c, v = fam.sparse(k)
            np.testing.assert_array_equal(r, ref[0])
            np.testing.assert_array_equal(c.astype(np.int32), ref[1])
            np.testing.assert_array_equal(v, ref[2])
            assert D[a, b] == dist
            cur.append((ref[0].astype(np.int32), ref[1].astype(np.int32), ref[2]))
            k += 1
    lens = [len(x) for x in seqs]
    for it in range(1, iters + 1):
        cur = orc.relax(lens, cur, qp=(w, 3.0, 1e-5 if it == iters else 0.01, seld, 6.0))
    fam.relax_qp(iters, w, seld, 6.0)
    for k in range(len(cur)):
        r, c, v = fam.sparse(k)
        np.testing.assert_array_equal(r, cur[k][0])
        np.testing.assert_array_equal(c.astype(np.int32), cur[k][1])
        np.testing.assert_array_equal(v, cur[k][2])
    fam.close()


def test_qp_cli_goldens_on_host_path():
    """The quickprobs binary's host path against the reference QuickProbs CLI
    (built from source): every golden family under the threshold."""
    runs = []
    for name, args in [('bb11028', []), ('bb11028', ['-c', '0']), ('bb11028', ['-c', '1', '-r', '5']),
                       ('div12', []), ('div12', ['-c', '0']), ('sim8', []), ('sim8', ['-c', '3', '-r', '50']),
                       ('qp_div60', []), ('qp_big210', [])]:
        fa = os.path.join(GOLDEN, 'cli', f'{name}.fa')
        tag = 'qp_' + name.replace('qp_', '') + ''.join('_' + a.strip('-') for a in args)
        if _cells(fa) <= HOST_MAX:
            runs.append((fa, args, os.path.join(GOLDEN, 'cli', f'{tag}.out')))
    for sub in ('real',):
        d = os.path.join(GOLDEN, sub)
        for f in sorted(os.listdir(d)):
            if f.endswith('.qp.out'):
                fa = os.path.join(d, f[:-len('.qp.out')] + '.fa')
                if _cells(fa) <= HOST_MAX:
                    runs.append((fa, [], os.path.join(d, f)))
    assert len(runs) >= 20, runs

    def one(r):
        fa, args, gold = r
        p = subprocess.run([QP_BIN, *args, fa], capture_output=True, timeout=300,
                           env=dict(os.environ, MLP_HOST_THREADS='2'))
        with open(gold, 'rb') as fh:
            return fa, args, p.returncode == 0 and p.stdout == fh.read()

    with ThreadPoolExecutor(4) as ex:
        bad = [(f, v) for f, v, ok in ex.map(one, runs) if not ok]
    assert not bad, bad


def test_qp_parity_sweep_on_host_path(tmp_path):
    """tools/parity_sweep.py's quickprobs half on every sweep family up to
    4e6 pair-cells (972 of the reference's TEST families): byte-identical."""
    out = tmp_path / 'sweep.txt'
    subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'parity_sweep.py'), str(out), '8', 'qp', '4e6'],
                   check=True, capture_output=True, timeout=1200)
    text = out.read_text()
    assert 'qp: 972/972 byte-identical' in text, text
    assert 'MISMATCH' not in text
