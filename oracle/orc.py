"""ctypes binding of oracle/_build/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker.  See oracle/oracle.h for the reference
lines each function restates.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

F32P = np.ctypeslib.ndpointer(np.float32, flags='C_CONTIGUOUS')
I32P = np.ctypeslib.ndpointer(np.int32, flags='C_CONTIGUOUS')
I64P = np.ctypeslib.ndpointer(np.int64, flags='C_CONTIGUOUS')


class Model(C.Structure):
    _fields_ = [
        ('initialDistribution', C.c_float * 5),
        ('transProb', C.c_float * 25),
        ('matchProb', C.c_float * 65536),
        ('insProb', C.c_float * 1280),
        ('local_transProb', C.c_float * 9),
        ('random_transProb', C.c_float * 2),
    ]


def build():
    subprocess.check_call(['make', '-s', '-C', _HERE, 'oracle'])


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, '_build', 'liboracle.so')
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.orc_model_init.argtypes = [C.POINTER(Model), C.c_float]
        L.orc_forward.argtypes = [C.POINTER(Model), C.c_char_p, C.c_int, C.c_char_p, C.c_int, C.c_int, F32P]
        L.orc_backward.argtypes = L.orc_forward.argtypes
        L.orc_total.argtypes = [C.POINTER(Model), C.c_char_p, C.c_int, C.c_char_p, C.c_int, F32P, F32P, C.c_int]
        L.orc_total.restype = C.c_float
        L.orc_posterior.argtypes = [C.POINTER(Model), C.c_char_p, C.c_int, C.c_char_p, C.c_int, F32P, F32P, C.c_int, F32P]
        L.orc_pf_posterior.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.c_int, F32P]
        L.orc_pair_posterior.argtypes = [C.POINTER(Model), C.c_char_p, C.c_int, C.c_char_p, C.c_int, C.c_int, F32P]
        L.orc_mea.argtypes = [C.c_int, C.c_int, F32P, C.c_char_p, C.POINTER(C.c_int)]
        L.orc_mea.restype = C.c_float
        L.orc_sparsify.argtypes = [C.c_int, C.c_int, F32P, I32P, C.c_void_p, C.c_void_p]
        L.orc_sparsify.restype = C.c_int64
        L.orc_relax.argtypes = [C.c_int, I32P, I64P, I64P, I32P, I32P, F32P, I32P, I64P, I32P, F32P, C.c_int64]
        L.orc_relax.restype = C.c_int64
        L.orc_viterbi.argtypes = [C.POINTER(Model), C.c_char_p, C.c_int, C.c_char_p, C.c_int, C.c_char_p, C.POINTER(C.c_int)]
        L.orc_viterbi.restype = C.c_float
        L.orc_model_adjustment.argtypes = [C.POINTER(Model), C.c_int, C.POINTER(C.c_char_p), I32P,
                                           C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.orc_pf_tables.argtypes = [np.ctypeslib.ndpointer(np.float64, flags='C_CONTIGUOUS'), I32P]
        L.orc_pair_loop.argtypes = [C.POINTER(Model), C.c_int, C.POINTER(C.c_char_p), I32P, C.c_int,
                                    C.c_int64, C.c_int, F32P, I64P]
        L.orc_pair_loop.restype = C.c_int64
        L.orc_qp_pair.argtypes = [C.POINTER(Model), C.c_char_p, C.c_int, C.c_char_p, C.c_int, F32P, F32P, F32P]
        L.orc_qp_pair.restype = C.c_float
        L.orc_qp_sparsify.argtypes = [C.c_int, C.c_int, F32P, I32P, C.c_void_p, C.c_void_p]
        L.orc_qp_sparsify.restype = C.c_int64
        L.orc_qp_relax.argtypes = [F32P, C.c_float, C.c_float] + L.orc_relax.argtypes
        L.orc_qp_relax.restype = C.c_int64
        L.orc_qp_relax_sel.argtypes = [F32P, C.c_float, C.c_float, F32P, C.c_float] + L.orc_relax.argtypes
        L.orc_qp_relax_sel.restype = C.c_int64
        U8P = np.ctypeslib.ndpointer(np.uint8, flags='C_CONTIGUOUS')
        U16P = np.ctypeslib.ndpointer(np.uint16, flags='C_CONTIGUOUS')
        F64P = np.ctypeslib.ndpointer(np.float64, flags='C_CONTIGUOUS')
        L.orc_relax_subset.argtypes = L.orc_relax.argtypes + [U8P]
        L.orc_relax_subset.restype = C.c_int64
        L.orc_pairs_csr.argtypes = [C.POINTER(Model), C.c_int, C.POINTER(C.c_char_p), I32P, C.c_int, I64P, C.c_int64,
                                    C.c_int, F32P, F32P, I32P, I64P, I32P, F32P, C.c_int64]
        L.orc_pairs_csr.restype = C.c_int64
        L.orc_csr_compare.argtypes = [C.c_int64, I32P, C.c_float, C.c_float, I64P, I64P, I32P, I32P, F32P,
                                      I64P, I64P, I32P, U16P, F32P, F64P]
        _LIB = L
    return _LIB


def model(delta=-1.0):
    m = Model()
    lib().orc_model_init(C.byref(m), float(delta))
    return m


def _s(seq):
    return b'@' + seq.encode()


def forward(m, s1, s2, flag):
    out = np.empty((5 if flag else 3) * (len(s1) + 1) * (len(s2) + 1), np.float32)
    lib().orc_forward(C.byref(m), _s(s1), len(s1), _s(s2), len(s2), int(flag), out)
    return out


def backward(m, s1, s2, flag):
    out = np.empty((5 if flag else 3) * (len(s1) + 1) * (len(s2) + 1), np.float32)
    lib().orc_backward(C.byref(m), _s(s1), len(s1), _s(s2), len(s2), int(flag), out)
    return out


def total(m, s1, s2, f, b, flag):
    return lib().orc_total(C.byref(m), _s(s1), len(s1), _s(s2), len(s2), f, b, int(flag))


def posterior(m, s1, s2, f, b, flag):
    out = np.empty((len(s1) + 1) * (len(s2) + 1), np.float32)
    lib().orc_posterior(C.byref(m), _s(s1), len(s1), _s(s2), len(s2), f, b, int(flag), out)
    return out


def pf_posterior(s1, s2):
    out = np.empty((len(s1) + 1) * (len(s2) + 1), np.float32)
    rc = lib().orc_pf_posterior(_s(s1), len(s1), _s(s2), len(s2), out)
    if rc:
        raise OverflowError('partition function overflow')
    return out


NPDO = 32  # pid flag: npdoAlign's ArrangePosteriorProbs pair body (oracle.h ORC_NPDO)


def pair_posterior(m, s1, s2, pid):
    out = np.empty((len(s1) + 1) * (len(s2) + 1), np.float32)
    lib().orc_pair_posterior(C.byref(m), _s(s1), len(s1), _s(s2), len(s2), int(pid), out)
    return out


def mea(L1, L2, post, with_path=False):
    if with_path:
        buf = C.create_string_buffer(L1 + L2 + 2)
        n = C.c_int(0)
        sc = lib().orc_mea(L1, L2, np.ascontiguousarray(post, np.float32), buf, C.byref(n))
        return sc, buf.raw[: n.value].decode()
    return lib().orc_mea(L1, L2, np.ascontiguousarray(post, np.float32), None, None)


def sparsify(L1, L2, post):
    post = np.ascontiguousarray(post, np.float32)
    rp = np.zeros(L1 + 2, np.int32)
    n = lib().orc_sparsify(L1, L2, post, rp, None, None)
    cols = np.empty(max(n, 1), np.int32)
    vals = np.empty(max(n, 1), np.float32)
    lib().orc_sparsify(L1, L2, post, rp, cols.ctypes.data, vals.ctypes.data)
    return rp, cols[:n], vals[:n]


def viterbi(m, s1, s2):
    buf = C.create_string_buffer(len(s1) + len(s2) + 2)
    n = C.c_int(0)
    sc = lib().orc_viterbi(C.byref(m), _s(s1), len(s1), _s(s2), len(s2), buf, C.byref(n))
    return sc, buf.raw[: n.value].decode()


def model_adjustment(m, seqs):
    arr = (C.c_char_p * len(seqs))(*[_s(s) for s in seqs])
    lens = np.array([len(s) for s in seqs], np.int32)
    ident = C.c_float(0)
    delta = C.c_float(0)
    vm = lib().orc_model_adjustment(C.byref(m), len(seqs), arr, lens, C.byref(ident), C.byref(delta))
    return vm, ident.value, delta.value


def pf_tables():
    sm = np.zeros((26, 26), np.float64)
    si = np.zeros(26, np.int32)
    lib().orc_pf_tables(sm, si)
    return sm, si


def pair_loop(m, seqs, pid, max_pairs=-1, threads=0):
    arr = (C.c_char_p * len(seqs))(*[_s(s) for s in seqs])
    lens = np.array([len(s) for s in seqs], np.int32)
    P = len(seqs) * (len(seqs) - 1) // 2
    if 0 <= max_pairs < P:
        P = max_pairs
    dist = np.zeros(max(P, 1), np.float32)
    nnz = np.zeros(max(P, 1), np.int64)
    tot = lib().orc_pair_loop(C.byref(m), len(seqs), arr, lens, int(pid), int(max_pairs), int(threads), dist, nnz)
    return dist[:P], nnz[:P], tot


def relax(lens, csrs, qp=None):
    """csrs: list over pairs (a<b row-major) of (rowptr[L_a+2], cols, vals).
    qp = (weights, selfweight, cutoff[, seldist, selectivity]): QuickProbs'
    consistency round instead (with its selectivity filter when seldist is given)."""
    N = len(lens)
    lens = np.asarray(lens, np.int32)
    row_off = np.zeros(len(csrs), np.int64)
    ent_off = np.zeros(len(csrs), np.int64)
    r = e = 0
    for p, (rp, c, v) in enumerate(csrs):
        row_off[p] = r
        ent_off[p] = e
        r += len(rp)
        e += len(c)
    in_rp = np.concatenate([c[0] for c in csrs]).astype(np.int32) if csrs else np.zeros(1, np.int32)
    in_c = np.concatenate([c[1] for c in csrs] + [np.zeros(1, np.int32)]).astype(np.int32)
    in_v = np.concatenate([c[2] for c in csrs] + [np.zeros(1, np.float32)]).astype(np.float32)
    out_rp = np.zeros_like(in_rp)
    out_off = np.zeros(max(len(csrs), 1), np.int64)
    cap = max(e, 1)
    out_c = np.zeros(cap, np.int32)
    out_v = np.zeros(cap, np.float32)
    if qp is None:
        tot = lib().orc_relax(N, lens, row_off, ent_off, in_rp, in_c, in_v, out_rp, out_off, out_c, out_v, cap)
    else:
        w = np.ascontiguousarray(qp[0], np.float32)
        if len(qp) > 3 and qp[3] is not None:
            d = np.ascontiguousarray(qp[3], np.float32)
            tot = lib().orc_qp_relax_sel(w, float(qp[1]), float(qp[2]), d, float(qp[4]), N, lens, row_off, ent_off,
                                         in_rp, in_c, in_v, out_rp, out_off, out_c, out_v, cap)
        else:
            tot = lib().orc_qp_relax(w, float(qp[1]), float(qp[2]), N, lens, row_off, ent_off, in_rp, in_c, in_v,
                                     out_rp, out_off, out_c, out_v, cap)
    assert tot >= 0
    res = []
    for p in range(len(csrs)):
        a = row_off[p]
        rp = out_rp[a: a + len(csrs[p][0])].copy()
        o = out_off[p]
        n = rp[-1]
        res.append((rp, out_c[o:o + n].copy(), out_v[o:o + n].copy()))
    return res


# ---- QuickProbs posterior stage (QP/Alignment/Multiple/PosteriorStage.cpp:123-196)
def qp_pair(m, s1, s2):
    """(hmm posterior, partition-function posterior, combined, distance)."""
    n = (len(s1) + 1) * (len(s2) + 1)
    h, g, p = (np.empty(n, np.float32) for _ in range(3))
    d = lib().orc_qp_pair(C.byref(m), _s(s1), len(s1), _s(s2), len(s2), h, g, p)
    return h, g, p, np.float32(d)


def qp_sparsify(L1, L2, post):
    """(row_ptr, cols, 16-bit fixed-point values) of entries >= 0.01."""
    post = np.ascontiguousarray(post, np.float32)
    rp = np.zeros(L1 + 2, np.int32)
    n = lib().orc_qp_sparsify(L1, L2, post, rp, None, None)
    cols = np.empty(max(n, 1), np.int32)
    q = np.empty(max(n, 1), np.uint16)
    lib().orc_qp_sparsify(L1, L2, post, rp, cols.ctypes.data, q.ctypes.data)
    return rp, cols[:n], q[:n]


# ---- bulk checkers (config-size parity tests and bench parity readouts)
def pair_index(n, a, b):
    return a * n - a * (a + 1) // 2 + (b - a - 1)


def pair_of(n, p):
    a = 0
    while p >= n - 1 - a:
        p -= n - 1 - a
        a += 1
    return a, a + 1 + p


def pairs_csr(m, seqs, pid, pairs, threads=0):
    """The pdoAlign pair body for a list of pairs (CPNP/MSA.cpp:939-1025):
    (dist, mea, rowptr, ent_off, cols, vals); rowptr holds L_a + 2 entries
    per listed pair (pair-local), ent_off len(pairs) + 1."""
    pairs = np.ascontiguousarray(pairs, np.int64)
    n = len(seqs)
    arr = (C.c_char_p * n)(*[_s(s) for s in seqs])
    lens = np.array([len(s) for s in seqs], np.int32)
    la = np.array([lens[pair_of(n, int(p))[0]] for p in pairs], np.int64)
    rp = np.zeros(max(int((la + 2).sum()), 1), np.int32)
    eo = np.zeros(len(pairs) + 1, np.int64)
    dist = np.zeros(max(len(pairs), 1), np.float32)
    mea_ = np.zeros(max(len(pairs), 1), np.float32)
    cap = int(sum(int(lens[pair_of(n, int(p))[0]]) * 64 for p in pairs)) + 1
    while True:
        cols = np.zeros(cap, np.int32)
        vals = np.zeros(cap, np.float32)
        tot = lib().orc_pairs_csr(C.byref(m), n, arr, lens, int(pid), pairs, len(pairs), int(threads), dist, mea_,
                                  rp, eo, cols, vals, cap)
        if tot >= 0:
            return dist[:len(pairs)], mea_[:len(pairs)], rp, eo, cols[:tot], vals[:tot]
        cap = int(eo[-1]) + 1


def store_view(lens, pairs, rowptr, ent_off):
    """Row/entry offsets of `pairs` inside a canonical store (include/mlpgpu.h
    layout): (L_a, row offsets, entry offsets)."""
    n = len(lens)
    lens = np.asarray(lens, np.int64)
    P = n * (n - 1) // 2
    a_of = np.repeat(np.arange(n), np.arange(n - 1, -1, -1))[:P]
    rp_off = np.zeros(P + 1, np.int64)
    rp_off[1:] = np.cumsum(lens[a_of] + 2)
    pairs = np.asarray(pairs, np.int64)
    return lens[a_of[pairs]].astype(np.int32), rp_off[pairs], np.asarray(ent_off, np.int64)[pairs]


def csr_compare(L1, ref, ours, rtol=1e-4, cutoff=0.01):
    """ref = (row offsets, entry offsets, rowptr int32, cols int32, vals);
    ours the same with uint16 cols.  Returns a dict of parity statistics
    (SURVEY.md section 8c rule)."""
    st = np.zeros(8, np.float64)
    lib().orc_csr_compare(len(L1), np.ascontiguousarray(L1, np.int32), float(rtol), float(cutoff),
                          *[np.ascontiguousarray(x) for x in ref], *[np.ascontiguousarray(x) for x in ours], st)
    keys = ('pairs', 'ref_entries', 'our_entries', 'common', 'max_rel_err', 'cutoff_flips', 'violations',
            'inexact')
    return {k: (float(v) if k == 'max_rel_err' else int(v)) for k, v in zip(keys, st)}


def relax_subset(lens, rowptr, ent_off, cols, vals, select):
    """orc_relax of the pairs with select[p] on a whole canonical store
    (flat arrays, include/mlpgpu.h layout).  Returns (rowptr, ent_off, cols,
    vals) of the output in the same layout (unselected pairs empty)."""
    n = len(lens)
    lens = np.asarray(lens, np.int32)
    P = n * (n - 1) // 2
    a_of = np.repeat(np.arange(n), np.arange(n - 1, -1, -1))[:P]
    row_off = np.zeros(P + 1, np.int64)
    row_off[1:] = np.cumsum(lens[a_of].astype(np.int64) + 2)
    eo = np.ascontiguousarray(ent_off, np.int64)
    in_rp = np.ascontiguousarray(rowptr, np.int32)
    in_c = np.ascontiguousarray(cols, np.int32) if len(cols) else np.zeros(1, np.int32)
    in_v = np.ascontiguousarray(vals, np.float32) if len(vals) else np.zeros(1, np.float32)
    sel = np.ascontiguousarray(select, np.uint8)
    out_rp = np.zeros_like(in_rp)
    out_off = np.zeros(max(P, 1), np.int64)
    idx = np.nonzero(sel)[0]
    cap = max(int((eo[idx + 1] - eo[idx]).sum()), 1)  # the output is masked to P_xy's entries
    out_c = np.zeros(cap, np.int32)
    out_v = np.zeros(cap, np.float32)
    tot = lib().orc_relax_subset(n, lens, row_off[:P], eo[:P], in_rp, in_c, in_v, out_rp, out_off, out_c, out_v,
                                 cap, sel)
    assert tot >= 0
    out_eo = np.zeros(P + 1, np.int64)
    out_eo[:P] = out_off[:P]
    out_eo[P] = tot
    return out_rp, out_eo, out_c[:tot], out_v[:tot]
