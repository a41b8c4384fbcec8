"""GPU parity: libmlpgpu (HIP, gfx950) against the reference golden vectors
(tests/golden/, produced by the reference's own objects) and against the CPU
oracle at larger sizes.  All calls go through the C ABI (include/mlpgpu.h).
"""
import os
import numpy as np
import pytest

import orc
from goldens import (GOLDEN, family_csrs, family_names, load_family, load_pair, load_qp_family, load_qp_pair,
                     pair_names, qp_family_csrs, qp_family_names, qp_pair_names)
from mlprobs_amd import synth
from mlprobs_amd.engine import PID_QP, Family
from parity import close_scalar, csr_close, csr_equal

pytestmark = pytest.mark.gpu

EXACT_PIDS = (2,)   # paths with no partition function: bit-exact


def _check_pair_csr(ref, ours, pid, what):
    if pid in EXACT_PIDS:
        csr_equal(ref, ours, what)
    else:
        csr_close(ref, ours, what=what)


@pytest.mark.parametrize('name', pair_names())
@pytest.mark.parametrize('pid', [0, 2, 3])
def test_pair_golden(name, pid):
    d = load_pair(name)
    fam = Family([d['s1'], d['s2']])
    fam.posteriors(pid, float(d['delta']))
    dist, mea, nnz = fam.results()
    ref = (d[f'pid{pid}.csr.rowptr'], d[f'pid{pid}.csr.cols'], d[f'pid{pid}.csr.vals'])
    _check_pair_csr(ref, fam.sparse(0), pid, f'{name} pid{pid}')
    ref_mea = d[f'pid{pid}.mea'][0]
    if pid in EXACT_PIDS:
        assert mea[0] == ref_mea
    else:
        assert close_scalar(ref_mea, mea[0])
    fam.close()


@pytest.mark.parametrize('name', family_names())
def test_family_golden(name):
    d = load_family(name)
    pid = int(d['pid'])
    fam = Family(d['seqs'])
    fam.posteriors(pid, float(d['delta']))
    D = fam.distances()
    n = len(d['seqs'])
    ref0 = family_csrs(d, 0)
    k = 0
    for a in range(n):
        for b in range(a + 1, n):
            _check_pair_csr(ref0[k], fam.sparse(k), pid, f'{name} p{k}')
            if pid in EXACT_PIDS:
                assert D[a, b] == d['distances'][a, b]
            else:
                assert close_scalar(d['distances'][a, b], D[a, b])
            k += 1
    fam.close()


@pytest.mark.parametrize('name', family_names())
def test_relax_golden(name):
    """Relaxation from the reference's own iteration-0 sparse set: bit-exact."""
    d = load_family(name)
    fam = Family(d['seqs'])
    ref0 = family_csrs(d, 0)
    rp = np.concatenate([c[0] for c in ref0]).astype(np.int32)
    eo = np.zeros(len(ref0) + 1, np.int64)
    eo[1:] = np.cumsum([len(c[1]) for c in ref0])
    cols = np.concatenate([c[1] for c in ref0] + [np.zeros(0, np.int32)]).astype(np.uint16)
    vals = np.concatenate([c[2] for c in ref0] + [np.zeros(0, np.float32)]).astype(np.float32)
    fam.import_csr(rp, eo, cols, vals)
    for it in range(1, int(d['reps']) + 1):
        fam.relax(1)
        ref = family_csrs(d, it)
        for k in range(len(ref)):
            csr_equal(ref[k], fam.sparse(k), f'{name} it{it} p{k}')
    fam.close()


@pytest.mark.parametrize('s,L,n,pid,seed', [(0.7, 120, 6, 2, 31), (0.5, 150, 5, 0, 32), (0.2, 130, 5, 3, 33),
                                             (0.7, 257, 3, 0, 34), (0.6, 64, 4, 2, 35), (0.6, 63, 4, 0, 36)])
def test_vs_oracle(s, L, n, pid, seed):
    fam_in = synth.family(n, L, s, seed=seed)
    seqs = [x for _, x in fam_in]
    delta = 0.132548
    m = orc.model(delta)
    fam = Family(seqs)
    fam.posteriors(pid, delta)
    D = fam.distances()
    k = 0
    for a in range(n):
        for b in range(a + 1, n):
            post = orc.pair_posterior(m, seqs[a], seqs[b], pid)
            ref = orc.sparsify(len(seqs[a]), len(seqs[b]), post)
            _check_pair_csr(ref, fam.sparse(k), pid, f'p{k}')
            sc = orc.mea(len(seqs[a]), len(seqs[b]), post)
            dist = np.float32(1) - np.float32(sc) / np.float32(min(len(seqs[a]), len(seqs[b])))
            if pid in EXACT_PIDS:
                assert D[a, b] == dist
            else:
                assert close_scalar(dist, D[a, b])
            k += 1
    # relaxation of our own posteriors vs the oracle's relaxation of the same input
    ours0 = [fam.sparse(k) for k in range(len(fam_in) * (len(fam_in) - 1) // 2)]
    ref1 = orc.relax([len(x) for x in seqs], [(r.astype(np.int32), c.astype(np.int32), v) for r, c, v in ours0])
    fam.relax(1)
    for k in range(len(ref1)):
        csr_equal(ref1[k], fam.sparse(k), f'relax p{k}')
    fam.close()


def _ragged_family(n, lo, hi, seed):
    rng = np.random.default_rng(seed)
    base = [x for _, x in synth.family(n, hi, 0.5, seed=seed)]
    return [x[: int(rng.integers(lo, hi + 1))] or 'A' for x in base]


def _check_family_vs_oracle(seqs, pid, tag):
    delta = 0.132548
    m = orc.model(delta)
    fam = Family(seqs)
    fam.posteriors(pid, delta)
    D = fam.distances()
    k = 0
    for a in range(len(seqs)):
        for b in range(a + 1, len(seqs)):
            post = orc.pair_posterior(m, seqs[a], seqs[b], pid)
            ref = orc.sparsify(len(seqs[a]), len(seqs[b]), post)
            _check_pair_csr(ref, fam.sparse(k), pid, f'{tag} p{k}')
            sc = orc.mea(len(seqs[a]), len(seqs[b]), post)
            dist = np.float32(1) - np.float32(sc) / np.float32(min(len(seqs[a]), len(seqs[b])))
            if pid in EXACT_PIDS:
                assert D[a, b] == dist, (tag, k)
            else:
                assert close_scalar(dist, D[a, b]), (tag, k)
            k += 1
    fam.close()


@pytest.mark.parametrize('pid', [2, 0])
def test_chains_many_short(pid):
    """Many short ragged pairs: chains of up to kChainMax members whose rows
    cross 64-row strips and member boundaries inside one strip."""
    _check_family_vs_oracle(_ragged_family(16, 2, 90, 41), pid, 'short')


def test_chains_long():
    """Long rows: W spans many 64-column boundary chunks."""
    _check_family_vs_oracle([x for _, x in synth.family(3, 900, 0.6, seed=42)], 2, 'long')


def test_chains_mixed_widths():
    """Column counts far apart: pairs go to different chains (width slack)."""
    seqs = _ragged_family(9, 150, 420, 43)
    _check_family_vs_oracle(seqs, 2, 'mixed')


@pytest.mark.parametrize('pid', [3, 0])
def test_pf_frames(pid):
    """Partition functions beyond fp64's range of one frame (2^200): runs of
    W (high self-score), near-identical long pairs (the real family
    oxx____8t2 that exposed a frame-label bug) and lengths that wrap several
    64-row strips; values must stay within the PF tolerance of the long-double
    oracle."""
    real = [x for _, x in synth.read_fasta(os.path.join(GOLDEN, 'real', 'oxx____8t2.fa'))]
    seqs = ['W' * 50, 'W' * 70, 'W' * 110, 'C' * 130, real[0], real[4], real[11], real[16]]
    _check_family_vs_oracle(seqs, pid, f'pf frames pid{pid}')


def test_batches_of_one(monkeypatch):
    """A scratch budget below one pair: every batch holds a single pair."""
    monkeypatch.setenv('MLP_SCRATCH_GB', '0.0001')
    _check_family_vs_oracle([x for _, x in synth.family(5, 70, 0.6, seed=44)], 2, 'batch1')


def test_pipelined_batches(monkeypatch):
    """Several batches alternating over the two posterior streams (all three
    models): compaction order, store growth and records stay pair-ordered."""
    monkeypatch.setenv('MLP_SCRATCH_GB', '0.004')
    _check_family_vs_oracle(_ragged_family(14, 60, 220, 45), 0, 'pipe')


# ---- family test: Viterbi alignments (CPNP/MSA.cpp:646-882)
@pytest.mark.parametrize('name', family_names())
def test_model_adjustment_golden(name):
    """pid class and delta from the reference's ModelAdjustmentTest (one thread)."""
    d = load_family(name)
    fam = Family(list(d['seqs']))
    ident, var, delta, code = fam.model_adjustment()
    assert code == int(d['variance_mean']), (name, ident, var, code)
    assert np.float32(delta) == np.float32(d['delta']), name
    fam.close()


@pytest.mark.parametrize('s,L,n,seed', [(0.6, 90, 6, 51), (0.3, 200, 4, 52), (0.8, 300, 3, 53)])
def test_viterbi_paths_vs_oracle(s, L, n, seed):
    seqs = _ragged_family(n, L // 3, L, seed)
    m = orc.model(0.132548)
    fam = Family(seqs)
    fam.viterbi(keep_paths=True)
    match, length = fam.viterbi_results()
    k = 0
    for a in range(n):
        for b in range(a + 1, n):
            _, ref = orc.viterbi(m, seqs[a], seqs[b])
            got = fam.viterbi_path(k)
            assert got == ref, (k, len(got), len(ref))
            assert length[k] == len(ref)
            i = j = 0
            same = 0
            for ch in ref:
                if ch == 'B':
                    same += seqs[a][i] == seqs[b][j]
                    i += 1
                    j += 1
                elif ch == 'X':
                    i += 1
                else:
                    j += 1
            assert match[k] == same
            k += 1
    fam.close()


@pytest.mark.parametrize('name', ['bb11028', 'div12', 'sim8'])
def test_family_features_cli_golden(name):
    """The `c_p_np_aln -G` line of the reference CLI (single thread)."""
    fa = os.path.join(GOLDEN, 'cli', f'{name}.fa')
    seqs = [x for _, x in synth.read_fasta(fa)]
    fam = Family(seqs)
    line = Family.features_line(fam.family_features(1.0))
    with open(os.path.join(GOLDEN, 'cli', f'{name}_G.out')) as fh:
        ref = fh.read().strip()
    assert line == ref, (line, ref)
    fam.close()


# small-class tiles (two workgroups per CU) whose staging area is too small
# for some outputs' images beside C: those are read in place from HBM on those
# z's (with and without passes over output subsets on the others)
_HBM_IMAGE_MODES = [{'MLP_TEST_RELAX_PATH': 'pairs', 'MLP_TEST_RELAX_SMALL_KB': '14', 'MLP_TEST_RELAX_GLOBAL_Z': '100000'},
                    {'MLP_TEST_RELAX_PATH': 'pairs', 'MLP_TEST_RELAX_SMALL_KB': '16', 'MLP_TEST_RELAX_GLOBAL_Z': '100000',
                     'MLP_TEST_RELAX_SPLIT_Z': '100000'}]


def _relax_both_paths(seqs, pid, iters, tag):
    """Tiled and row-task relaxation vs the oracle, bit-exact, `iters` rounds."""
    n = len(seqs)
    fam = Family(seqs)
    fam.posteriors(pid, 0.132548)
    rp, eo, cols, vals = [a.copy() for a in fam.export()]
    cur = [fam.sparse(k) for k in range(n * (n - 1) // 2)]
    cur = [(r.astype(np.int32), c.astype(np.int32), v) for r, c, v in cur]
    lens = [len(x) for x in seqs]
    refs = []
    for _ in range(iters):
        cur = orc.relax(lens, cur)
        refs.append(cur)
    # tiled kernel with up to 4 outputs per tile, one output per tile, the
    # large-prefetch instantiation, and the row-task kernel
    # and tiles over a 48 KB staging area whose oversize z's are staged in
    # passes over subsets of the outputs (MLP_TEST_RELAX_SPLIT_Z: no limit), and
    # small-class tiles over a tiny staging area, whose outputs' images are
    # read in place from HBM on the z's where they do not fit beside C
    modes = [{'MLP_TEST_RELAX_PATH': 'pairs'}, {'MLP_TEST_RELAX_PATH': 'pairs', 'MLP_TEST_RELAX_TILE': '1'},
             {'MLP_TEST_RELAX_PATH': 'pairs', 'MLP_TEST_RELAX_KP': '9'}, {'MLP_TEST_RELAX_PATH': 'tasks'},
             {'MLP_TEST_RELAX_LDS_KB': '48', 'MLP_TEST_RELAX_SPLIT_Z': '100000'}] + _HBM_IMAGE_MODES
    for env in modes:
        os.environ.update(env)
        try:
            fam.import_csr(rp, eo, cols, vals)
            for it in range(iters):
                fam.relax(1)
                for k in range(len(refs[it])):
                    csr_equal(refs[it][k], fam.sparse(k), f'{tag} {env} it{it + 1} p{k}')
        finally:
            for key in env:
                del os.environ[key]
    fam.close()


def test_relax_pair_path_divergent():
    seqs = [x for _, x in synth.family(40, 150, 0.7, seed=41)]
    _relax_both_paths(seqs, 0, 2, 'div')


def test_relax_pair_path_ragged():
    # lengths 1..400: idle waves, images of very different sizes, empty rows
    seqs = _ragged_family(24, 1, 400, 42)
    _relax_both_paths(seqs, 1, 2, 'ragged')


def test_relax_pair_path_similar():
    seqs = [x for _, x in synth.family(30, 200, 0.2, seed=43)]
    _relax_both_paths(seqs, 3, 3, 'similar')


def test_relax_hbm_images_exercised(capfd):
    """Small-class tiles whose outputs' images are read in place from HBM on
    the z's where they do not fit beside C (relax.hip, bit 12 + t of the z
    schedule): the plan log must show such outputs for some staging size, and
    one round must equal the oracle's bit for bit."""
    seqs = _ragged_family(24, 1, 400, 42)
    n = len(seqs)
    fam = Family(seqs)
    fam.posteriors(1, 0.132548)
    rp, eo, cols, vals = [a.copy() for a in fam.export()]
    cur = [fam.sparse(k) for k in range(n * (n - 1) // 2)]
    ref = orc.relax([len(x) for x in seqs], [(r.astype(np.int32), c.astype(np.int32), v) for r, c, v in cur])
    seen = 0
    for kb in (14, 16, 20, 24, 32):
        env = {'MLP_TEST_RELAX_PATH': 'pairs', 'MLP_TEST_RELAX_SMALL_KB': str(kb), 'MLP_TEST_RELAX_GLOBAL_Z': '100000',
               'MLP_LOG_PLAN': '1'}
        os.environ.update(env)
        try:
            fam.import_csr(rp, eo, cols, vals)
            fam.relax(1)
            fam.synchronize()
            for k in range(len(ref)):
                csr_equal(ref[k], fam.sparse(k), f'hbm {kb} KB p{k}')
        finally:
            for key in env:
                del os.environ[key]
        err = capfd.readouterr().err
        got = [int(l.split('hbm-image outputs')[1]) for l in err.splitlines() if 'hbm-image outputs' in l]
        assert got, err
        seen += sum(got)
    fam.close()
    assert seen > 0


def test_relax_blockmfma_eval():
    """The dense-block MFMA evaluation variant (relax_mfma.hip): fused
    products, so held to SURVEY 8c's 1e-4 relative rule against a
    double-precision sum over the same blocks, not to bit identity."""
    seqs = [x for _, x in synth.family(24, 150, 0.7, seed=44)]
    fam = Family(seqs)
    fam.posteriors(0, 0.0)
    r = fam.relax_blockmfma_eval([0, 1, 2, 5], [7, 9, 20, 23])
    fam.close()
    assert r['outputs'] == 16 and r['cells_checked'] > 100 and r['dense_macs'] > 0
    assert r['max_rel_err'] < 1e-4, r


# ---- QuickProbs posterior stage (QP/Alignment/Multiple/PosteriorStage.cpp:123-196)
def _qp_expected(seqs, a, b):
    """Oracle CSR (values as QuickProbs reads its 16-bit entries) and distance."""
    h, g, p, dist = orc.qp_pair(orc.model(-1.0), seqs[a], seqs[b])
    rp, cols, q = orc.qp_sparsify(len(seqs[a]), len(seqs[b]), p)
    return (rp, cols, q.astype(np.float32) / np.float32(65535)), dist


def _check_qp_family(seqs, tag):
    n = len(seqs)
    fam = Family(seqs)
    fam.posteriors(PID_QP, 0.0)
    D = fam.distances()
    k = 0
    for a in range(n):
        for b in range(a + 1, n):
            ref, dist = _qp_expected(seqs, a, b)
            csr_equal(ref, fam.sparse(k), f'{tag} qp p{k}')
            assert D[a, b] == dist, (tag, k, D[a, b], dist)
            k += 1
    fam.close()


@pytest.mark.parametrize('name', qp_pair_names())
def test_qp_golden(name):
    """Bit-exact against the reference QuickProbs build: the sparse rows, the
    16-bit values and the distance of every golden pair."""
    d = load_qp_pair(name)
    fam = Family([d['s1'], d['s2']])
    fam.posteriors(PID_QP, 0.0)
    ref = (d['row_ptr'], d['cols'], d['qvals'].astype(np.float32) / np.float32(65535))
    csr_equal(ref, fam.sparse(0), f'qp {name}')
    assert fam.distances()[0, 1] == d['dist'][0]
    fam.close()


@pytest.mark.parametrize('s,L,n,seed', [(0.7, 150, 6, 61), (0.4, 220, 5, 62), (0.15, 180, 4, 63)])
def test_qp_vs_oracle(s, L, n, seed):
    _check_qp_family([x for _, x in synth.family(n, L, s, seed=seed)], f'qp{seed}')


def test_qp_ragged_chains():
    """Many short ragged pairs stacked into chains, lengths 1..260."""
    _check_qp_family(_ragged_family(12, 1, 260, 64), 'qp_ragged')


# ---- QuickProbs consistency (QP/Alignment/Multiple/ConsistencyStage.cpp:90-258)
_RELAX_MODES = [{'MLP_TEST_RELAX_PATH': 'pairs'}, {'MLP_TEST_RELAX_PATH': 'pairs', 'MLP_TEST_RELAX_TILE': '1'},
                {'MLP_TEST_RELAX_PATH': 'pairs', 'MLP_TEST_RELAX_KP': '9'}, {'MLP_TEST_RELAX_PATH': 'tasks'}] + _HBM_IMAGE_MODES


def _import(fam, csrs):
    rp = np.concatenate([c[0] for c in csrs]).astype(np.int32)
    eo = np.zeros(len(csrs) + 1, np.int64)
    eo[1:] = np.cumsum([len(c[1]) for c in csrs])
    cols = np.concatenate([c[1] for c in csrs] + [np.zeros(0, np.int32)]).astype(np.uint16)
    vals = np.concatenate([c[2] for c in csrs] + [np.zeros(0, np.float32)]).astype(np.float32)
    fam.import_csr(rp, eo, cols, vals)


@pytest.mark.parametrize('name', qp_family_names())
def test_qp_relax_golden(name):
    """QuickProbs' consistency rounds from the reference's own posterior-stage
    set, bit-exact against the reference build, on every relaxation path."""
    d = load_qp_family(name)
    ref = qp_family_csrs(d, d['iters'])
    fam = Family(d['seqs'])
    for env in _RELAX_MODES:
        os.environ.update(env)
        try:
            _import(fam, qp_family_csrs(d, 0))
            n = len(d['seqs'])
            fam.relax_qp(d['iters'], d['weights'], d['seldist'].reshape(n, n), float(d['selectivity'][0]))
            for k in range(len(ref)):
                csr_equal(ref[k], fam.sparse(k), f'{name} {env} p{k}')
        finally:
            for key in env:
                del os.environ[key]
    fam.close()


@pytest.mark.parametrize('n,L,s,iters,seed,sel', [(9, 140, 0.6, 2, 71, False), (7, 200, 0.3, 1, 72, False),
                                                  (12, 90, 0.7, 3, 73, False), (14, 120, 0.6, 2, 74, True),
                                                  (10, 260, 0.5, 1, 75, True)])
def test_qp_stage_vs_oracle(n, L, s, iters, seed, sel):
    """QuickProbs posterior stage then consistency, all on the GPU, against the
    oracle's restatement of both stages; `sel`: with a subtree-size-like
    selectivity matrix that rejects z (ExtendedMSA.cpp:96-100, threshold 6)."""
    seqs = [x for _, x in synth.family(n, L, s, seed=seed)]
    rng = np.random.default_rng(seed)
    w = rng.uniform(1, 30, n).astype(np.float32)
    seld = None
    if sel:
        seld = rng.integers(2, n + 1, (n, n)).astype(np.float32)
        seld = np.minimum(seld, seld.T)
        np.fill_diagonal(seld, 0)
    fam = Family(seqs)
    fam.posteriors(PID_QP, 0.0)
    cur = [_qp_expected(seqs, a, b)[0] for a in range(n) for b in range(a + 1, n)]
    cur = [(r.astype(np.int32), c.astype(np.int32), v) for r, c, v in cur]
    lens = [len(x) for x in seqs]
    for it in range(1, iters + 1):
        cur = orc.relax(lens, cur, qp=(w, 3.0, 1e-5 if it == iters else 0.01, seld, 6.0))
    fam.relax_qp(iters, w, seld, 6.0)
    for k in range(len(cur)):
        csr_equal(cur[k], fam.sparse(k), f'qp stage p{k}')
    fam.close()


def _gapped(rng, s, L):
    """s with gaps inserted at random to length L, and its getMapping array."""
    pos = np.sort(rng.choice(np.arange(1, L + 1), size=len(s), replace=False))
    row = ['-'] * (L + 1)
    for k, c in zip(pos, s):
        row[k] = c
    return ''.join(row[1:]), np.concatenate([[0], pos]).astype(np.int32)


def _pair(n, a, b):
    return a * n - a * (a + 1) // 2 + (b - a - 1)


def _profile_case(seed, n, L, sub, A, B, env=None, mea=True, pad1=9, pad2=5):
    """mlp_profile_posterior (QuickProbs' buildPosterior on the GPU) against a
    plain restatement of ParallelProbabilisticModel.cpp:301-430 over the same
    relaxed sparse set: weights in double cast to float, terms in (i, j, row,
    entry) order, w * v then +=; bit-exact."""
    rng = np.random.default_rng(seed)
    seqs = [x for _, x in synth.family(n, L, sub, seed=seed)]
    fam = Family(seqs)
    fam.posteriors(PID_QP, 0.0)
    w = rng.uniform(0.01, 0.3, n).astype(np.float32)
    fam.relax_qp(2, w)
    need = set(A) | set(B)
    dense = {}  # dense views of the ordered blocks the profiles use
    for a in range(n):
        for b in range(a + 1, n):
            if not ((a in A and b in B) or (a in B and b in A)):
                continue
            rp, c, v = fam.sparse(_pair(n, a, b))
            rows = [[] for _ in range(len(seqs[a]) + 1)]
            trows = [[] for _ in range(len(seqs[b]) + 1)]
            for i in range(1, len(seqs[a]) + 1):
                for e in range(rp[i], rp[i + 1]):
                    rows[i].append((int(c[e]), float(v[e])))
                    trows[int(c[e])].append((i, float(v[e])))
            dense[(a, b)] = rows
            dense[(b, a)] = trows
    assert need
    L1 = max(len(seqs[k]) for k in A) + pad1
    L2 = max(len(seqs[k]) for k in B) + pad2
    mA = [_gapped(rng, seqs[k], L1)[1] for k in A]
    mB = [_gapped(rng, seqs[k], L2)[1] for k in B]
    old = {k: os.environ.get(k) for k in (env or {})}
    try:
        os.environ.update(env or {})
        got = fam.profile_posterior(w, A, mA, L1, B, mB, L2)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    ref = np.zeros((L1 + 1, L2 + 1), np.float32)
    total = 0.0
    for a in A:
        for b in B:
            total += float(w[a]) * float(w[b])
    for ia, a in enumerate(A):
        for jb, b in enumerate(B):
            wf = np.float32((float(w[a]) * float(w[b])) / total)
            rows = dense[(a, b)]
            for ii in range(1, len(seqs[a]) + 1):
                r = mA[ia][ii]
                for col, v in rows[ii]:
                    c = mB[jb][col]
                    ref[r, c] = np.float32(ref[r, c] + np.float32(wf * np.float32(v)))
    np.testing.assert_array_equal(got, ref)
    if mea:
        # the same matrix left on the device: MEA there, and a gather
        fam.profile_defer(True)
        fam.profile_posterior(w, A, mA, L1, B, mB, L2)
        path, score = fam.profile_mea(L1, L2)
        rpath, rscore = _mea_ref(ref)
        assert path == rpath and score == rscore, (score, rscore)
        cells = np.array([0, L2 + 2, (L1 + 1) * (L2 + 1) - 1, 3 * (L2 + 1) + 5], np.int64)
        np.testing.assert_array_equal(fam.profile_gather(cells), ref.reshape(-1)[cells])
        fam.profile_defer(False)
    fam.close()


def _mea_ref(post):
    """ComputeAlignment (ProbabilisticModel.h:804-864) in float32, serially."""
    L1, L2 = post.shape[0] - 1, post.shape[1] - 1
    old = np.zeros(L2 + 1, np.float32)
    tb = np.zeros((L1 + 1, L2 + 1), np.int8)
    for i in range(1, L1 + 1):
        new = np.zeros(L2 + 1, np.float32)
        for j in range(1, L2 + 1):
            x1 = np.float32(post[i, j] + old[j - 1])
            x2, x3 = new[j - 1], old[j]
            if x1 >= x2:
                v, b = (x1, 0) if x1 >= x3 else (x3, 2)
            elif x2 >= x3:
                v, b = x2, 1
            else:
                v, b = x3, 2
            new[j] = v
            tb[i, j] = b
        old = new
    r, c, out = L1, L2, []
    while r or c:
        b = 1 if r == 0 else 2 if c == 0 else tb[r, c]
        if b == 1:
            c -= 1
            out.append('Y')
        elif b == 2:
            r -= 1
            out.append('X')
        else:
            r -= 1
            c -= 1
            out.append('B')
    return ''.join(reversed(out)), old[L2]


@pytest.mark.parametrize('seed', [81, 82])
def test_profile_posterior_vs_restatement(seed):
    _profile_case(seed, 9, 70, 0.5, [0, 3, 5, 8], [1, 2, 6])


@pytest.mark.parametrize('stage,split', [('8', None), ('24', '3'), ('1', '2'), (None, '5')])
def test_profile_posterior_stage_branches(stage, split):
    """k_profile_post's rarer paths on small profiles: a stage smaller than
    one row (the piecewise long-row branch), runs cut short by the stage
    (fewer than 64 pairs), and forced column ranges per row."""
    env = {}
    if stage:
        env['MLP_TEST_PROFILE_STAGE'] = stage
    if split:
        env['MLP_TEST_PROFILE_SPLIT'] = split
    _profile_case(83, 9, 70, 0.7, [0, 3, 5, 8], [1, 2, 6], env)


def test_profile_mea_multi_strip():
    """Device MEA over profiles of ~190 x ~185 columns (three 64-row strips)."""
    _profile_case(86, 12, 180, 0.5, [0, 2, 4, 7, 9], [1, 3, 11])


def test_profile_mea_groups():
    """~1150 profile-A columns: 18 strips, each polling the row the one
    above hands off (NaN-filled rows, mlp_profile_mea)."""
    _profile_case(87, 4, 140, 0.5, [0, 1], [2, 3], pad1=1010)


def test_profile_mea_wide_rows():
    """~4150 profile-B columns: rows of ~65 blocks, so a poll's 64 columns
    serve up to four blocks many times over."""
    _profile_case(88, 4, 140, 0.5, [0, 1], [2, 3], pad2=4010)


def _mea_matrix(rng, L1, L2, kind):
    post = np.zeros((L1 + 1, L2 + 1), np.float32)
    body = post[1:, 1:]
    if kind == 'dense':
        body[:] = rng.uniform(0, 1, body.shape)
    elif kind == 'sparse':   # a refinement's profile posterior: few entries, many exact ties
        k = max(1, body.size // 600)
        body.reshape(-1)[rng.choice(body.size, k, replace=False)] = rng.uniform(0.01, 8, k)
    elif kind == 'tails':    # entries in each row's first and last 16 columns only
        w = min(16, L2)
        body[:, :w] = rng.uniform(0, 1, (L1, w)) * (rng.uniform(0, 1, (L1, w)) < 0.3)
        body[:, L2 - w:] = rng.uniform(0, 1, (L1, w)) * (rng.uniform(0, 1, (L1, w)) < 0.3)
    elif kind == 'band':
        for i in range(L1):
            j = int(i * L2 / L1)
            body[i, max(0, j - 3):j + 4] = rng.uniform(0.01, 1, len(range(max(0, j - 3), min(L2, j + 4))))
    return post   # 'zeros': every cell a tie


@pytest.mark.parametrize('L1,L2,kind', [
    (1, 1, 'dense'), (1, 300, 'sparse'), (40, 1, 'dense'), (50, 16, 'tails'), (64, 64, 'dense'),
    (65, 17, 'tails'), (128, 128, 'band'), (128, 200, 'tails'), (130, 300, 'zeros'), (200, 63, 'sparse'),
    (261, 8076, 'sparse'), (261, 2000, 'tails'), (700, 900, 'dense'), (1100, 700, 'tails'), (2000, 600, 'band')])
def test_profile_mea_any_matrix(L1, L2, kind):
    """Device MEA (mlp_profile_set + mlp_profile_mea) of arbitrary matrices
    against the oracle's ComputeAlignment (orc_mea, ProbabilisticModel.h:
    804-864): path and score bit for bit.  'tails' puts entries where a strip's
    first blocks read past their rows (round 5: the fourth block's lanes at
    columns <= 0 went unmasked and read the row before's last columns -- a
    C2 -p 1 refinement diverged from the reference); 'sparse' / 'zeros' are
    tie-heavy."""
    rng = np.random.default_rng(L1 * 7919 + L2)
    post = _mea_matrix(rng, L1, L2, kind)
    fam = Family([x for _, x in synth.family(3, 20, 0.5, seed=1)])
    try:
        fam.profile_set(post)
        path, score = fam.profile_mea(L1, L2)
        rscore, rpath = orc.mea(L1, L2, post, with_path=True)
        assert score == np.float32(rscore), (score, rscore)
        assert path == rpath
        cells = np.array([0, L2 + 2, (L1 + 1) * (L2 + 1) - 1], np.int64)
        np.testing.assert_array_equal(fam.profile_gather(cells), post.reshape(-1)[cells])
    finally:
        fam.close()


def test_profile_set_rejects_non_posteriors():
    """mlp_profile_set takes finite entries >= +0 only (the device MEA polls
    for non-NaN hand-offs and its choices assume that range): NaN, -0, a
    negative value or infinity is MLP_ERR_ARG, and a valid matrix still works."""
    fam = Family([x for _, x in synth.family(3, 20, 0.5, seed=1)])
    try:
        for bad in (np.nan, -0.0, -1e-30, np.inf):
            post = np.zeros((6, 9), np.float32)
            post[3, 4] = bad
            with pytest.raises(RuntimeError, match='bad argument'):
                fam.profile_set(post)
        post = np.zeros((6, 9), np.float32)
        post[1:, 1:] = 0.25
        fam.profile_set(post)
        path, score = fam.profile_mea(5, 8)
        assert score == np.float32(orc.mea(5, 8, post, with_path=True)[0])
    finally:
        fam.close()


def test_profile_posterior_many_sequences():
    """More than 64 sequences in profile A: the column compaction runs in
    several 64-sequence chunks (and with a small stage, partial runs)."""
    _profile_case(84, 72, 30, 0.5, list(range(0, 72, 1))[:66], [66, 68, 71])
    _profile_case(85, 72, 30, 0.5, list(range(3, 72))[:67], [0, 1], {'MLP_TEST_PROFILE_STAGE': '40'})


# ---- npdoAlign's pair body (MLP_PID_NPDO: ArrangePosteriorProbs,
# CPNP/MSA.cpp:1636-1765): the RMS terms in its order and the distance
# score / #B, #B carried along the MEA recurrence on the GPU
@pytest.mark.parametrize('name', ['div12', 'sim8', 'bb11028'])
def test_npdo_golden(name):
    """Against the reference's own ArrangePosteriorProbs (ref_probe npdo,
    tests/golden/gen_np.py) at the family's pid / delta."""
    g = np.load(os.path.join(GOLDEN, f'np_pairs_{name}.npz'))
    seqs = [s for _, s in synth.read_fasta(os.path.join(GOLDEN, 'cli', f'{name}.fa'))]
    pid = int(g['pid'])
    fam = Family(seqs)
    fam.posteriors(pid | NPDO, float(g['delta']))
    dist = fam.results()[0]
    for k in range(len(g['ab'])):
        la = int(g['L1'][k])
        r0 = int(g['eoff'][k])
        rp = g['rp'][sum(int(x) + 2 for x in g['L1'][:k]):][:la + 2]
        ref = (rp, g['cols'][r0:r0 + rp[-1]], g['vals'][r0:r0 + rp[-1]])
        _check_pair_csr(ref, fam.sparse(k), pid, f'{name} p{k}')
        if pid in EXACT_PIDS:
            assert dist[k] == g['dist'][k]
        else:
            assert close_scalar(g['dist'][k], dist[k]), (name, k)
    fam.close()


NPDO = 32


@pytest.mark.parametrize('s,L,n,pid,seed', [(0.7, 150, 5, 2, 91), (0.6, 260, 4, 2, 92), (0.5, 200, 5, 0, 93),
                                             (0.2, 130, 4, 3, 94)])
def test_npdo_vs_oracle(s, L, n, pid, seed):
    """Rows cross 64-row strips (the #B count rides the strip boundary row);
    pid 2 bit-exact (no partition function), else the section 8c rule."""
    seqs = _ragged_family(n, L // 2, L, seed)
    delta = 0.132548
    fam = Family(seqs)
    fam.posteriors(pid | NPDO, delta)
    m = orc.model(delta)
    pairs = np.arange(fam.npairs)
    dist, _, rp, eo, cols, vals = orc.pairs_csr(m, seqs, pid | orc.NPDO, pairs)
    g = fam.results()[0]
    roff = 0
    for k in pairs:
        a, b = orc.pair_of(n, int(k))
        la = len(seqs[a])
        ref = (rp[roff:roff + la + 2], cols[eo[k]:eo[k + 1]], vals[eo[k]:eo[k + 1]])
        roff += la + 2
        _check_pair_csr(ref, fam.sparse(int(k)), pid, f'p{k}')
        if pid in EXACT_PIDS:
            assert g[k] == dist[k], (k, g[k], dist[k])
        else:
            assert close_scalar(dist[k], g[k]), k
    fam.close()


def test_pf_long_double_overflow():
    """The reference stops ("huge val error", exit 1) once a partition-function
    value reaches long double infinity (CPNP/MSAPartProbs.cpp:547-589); the
    oracle (x87 long double) overflows between 3400 and 3700 identical W
    residues.  The GPU's fp64 frames reach much further, so it flags the same
    bound: MLP_ERR_OVERFLOW at 3800, a normal result at 3300."""
    from mlprobs_amd.engine import MlpError
    ok = Family(['W' * 3300, 'W' * 3300])
    ok.posteriors(3, 0.132548)
    assert ok.results()[2][0] > 0
    ok.close()
    with pytest.raises(OverflowError):
        orc.pf_posterior('W' * 3800, 'W' * 3800)
    big = Family(['W' * 3800, 'W' * 3800])
    with pytest.raises(MlpError) as e:
        big.posteriors(3, 0.132548)
    assert e.value.code == 3
    big.close()


def test_pf_posterior_in_zm_slot_bit_identical():
    """Under a small scratch budget the PF posterior is written into the low
    half of its cell's consumed PF forward Zm slot (mlp_posteriors, <= 48 GB);
    the sparse store, distances and MEA scores must be the same bytes as with
    its own array (the default budget), over several batches."""
    seqs = _ragged_family(24, 80, 260, 46)
    outs = []
    for budget in (None, 64 << 20):
        fam = Family(seqs)
        if budget:
            assert fam._L.mlp_set_scratch(fam._ctx, budget) == 0
        fam.posteriors(0, 0.132548)
        outs.append([np.ascontiguousarray(a).tobytes() for a in (*fam.export(), *fam.results())])
        fam.close()
    assert outs[0] == outs[1]
