"""Python mirror of the C_P_NP_Aln posterior / consistency interface, running
on the MI355X through libmlpgpu's C ABI (include/mlpgpu.h).

Reference interface (kuangmeng/MLProbs baseMSA/C_P_NP_Aln):
  - pdoAlign pair loop (CPNP/MSA.cpp:927-1032): per pair posterior, distance
    1 - MEA/min(L_a, L_b), SparseMatrix (>= 0.01)   -> Family.posteriors()
  - MSA::DoRelaxation x numConsistencyReps (CPNP/MSA.cpp:1041-1051)
                                                    -> Family.relax()
  - SparseMatrix rows/columns (CPNP/SparseMatrix.h) -> Family.sparse(a, b)

There is deliberately no CPU fallback: if the HIP library is missing or no
GPU is visible every entry point raises.
"""
import ctypes as C
import os

import numpy as np

from . import build as _build

_LIB = None

I64 = C.c_int64
F32P = np.ctypeslib.ndpointer(np.float32, flags='C_CONTIGUOUS')
I32P = np.ctypeslib.ndpointer(np.int32, flags='C_CONTIGUOUS')
I64P = np.ctypeslib.ndpointer(np.int64, flags='C_CONTIGUOUS')
U16P = np.ctypeslib.ndpointer(np.uint16, flags='C_CONTIGUOUS')

PID_QP = 16  # include/mlpgpu.h MLP_PID_QP: QuickProbs' posterior stage
ERRORS = {1: 'bad argument', 2: 'HIP error', 3: 'partition function overflow', 4: 'state error',
          5: 'RCCL error', 6: 'device memory'}
KERNELS = ['forward', 'backward', 'local_totals', 'merge_mea_sparsify', 'compact', 'relax',
           'transpose', 'filter', 'allgather', 'viterbi']


class MlpError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f'{ERRORS.get(code, code)}: {msg}')
        self.code = code


def lib_path():
    return _build.LIB


def lib():
    """Load libmlpgpu.so (in-tree).  Raises if it is missing."""
    global _LIB
    if _LIB is None:
        var = os.environ.get('MLP_LIB_VARIANT')
        path = _build.variant_path(var) if var else _build.LIB
        if not os.path.exists(path):
            raise RuntimeError(f'{path} missing: run `python -m mlprobs_amd.build` (hipcc, gfx950)')
        L = C.CDLL(path)
        P = C.c_void_p
        L.mlp_ctx_create.argtypes = [C.c_int, C.POINTER(P)]
        L.mlp_ctx_destroy.argtypes = [P]
        L.mlp_ctx_destroy.restype = None
        L.mlp_last_error.argtypes = [P]
        L.mlp_last_error.restype = C.c_char_p
        L.mlp_set_scratch.argtypes = [P, C.c_uint64]
        L.mlp_family_load.argtypes = [P, C.c_int, C.c_char_p, I64P]
        L.mlp_family_npairs.argtypes = [P]
        L.mlp_family_npairs.restype = I64
        L.mlp_posteriors.argtypes = [P, C.c_int, C.c_float, I64, I64]
        L.mlp_pair_results.argtypes = [P, I64, I64, C.c_void_p, C.c_void_p, C.c_void_p]
        L.mlp_csr_total.argtypes = [P, C.POINTER(I64)]
        L.mlp_csr_export.argtypes = [P, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.mlp_csr_import.argtypes = [P, I32P, I64P, U16P, F32P]
        L.mlp_relax.argtypes = [P, C.c_int]
        L.mlp_relax_range.argtypes = [P, I64, I64]
        L.mlp_relax_qp.argtypes = [P, C.c_int, F32P]
        L.mlp_relax_qp_selective.argtypes = [P, C.c_int, F32P, C.c_void_p, C.c_float]
        L.mlp_profile_posterior.argtypes = [P, F32P, C.c_int, I32P, C.c_int, I32P, C.c_int, I32P, C.c_int, I32P,
                                            F32P]
        L.mlp_profile_posterior_cpnp.argtypes = [P, C.c_void_p, C.c_int, I32P, C.c_int, I32P, C.c_int, I32P, C.c_int,
                                                 I32P, F32P]
        L.mlp_viterbi.argtypes = [P, I64, I64, C.c_int]
        L.mlp_viterbi_results.argtypes = [P, I64, I64, C.c_void_p, C.c_void_p]
        L.mlp_viterbi_path.argtypes = [P, I64, C.c_void_p, C.c_void_p]
        L.mlp_model_adjustment.argtypes = [P, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.mlp_family_features.argtypes = [P, C.c_float, C.c_void_p, C.c_void_p]
        L.mlp_comm_unique_id.argtypes = [C.c_char_p]
        L.mlp_comm_init.argtypes = [P, C.c_char_p, C.c_int, C.c_int]
        L.mlp_shard_range.argtypes = [P, C.c_int, C.c_int, C.POINTER(I64), C.POINTER(I64)]
        L.mlp_shard_plan.argtypes = [C.c_int, I32P, C.c_int, C.c_int, C.POINTER(I64), C.POINTER(I64)]
        L.mlp_gather_layout.argtypes = [C.c_int, I64, I64P, I64P]
        L.mlp_allgather.argtypes = [P]
        L.mlp_synchronize.argtypes = [P]
        L.mlp_profile.argtypes = [P, C.c_int]
        L.mlp_profile_reset.argtypes = [P]
        L.mlp_kernel_times.argtypes = [P, C.c_void_p, C.c_void_p, C.c_void_p]
        L.mlp_ctx_create_mask.argtypes = [C.c_uint64, C.POINTER(P)]
        L.mlp_ctx_create_host.argtypes = [C.POINTER(P)]
        L.mlp_ctx_is_host.argtypes = [P]
        L.mlp_set_shards.argtypes = [P, C.c_int]
        L.mlp_shard_count.argtypes = [P]
        L.mlp_relax_shard_plan.argtypes = [C.c_int, I32P, I64P, C.c_int, I64P]
        L.mlp_relax_blockmfma_eval.argtypes = [P, C.c_int, I32P, C.c_int, I32P, C.c_void_p]
        L.mlp_profile_defer.argtypes = [P, C.c_int]
        L.mlp_profile_mea.argtypes = [P, C.c_char_p, C.POINTER(C.c_int32), C.POINTER(C.c_float)]
        L.mlp_profile_gather.argtypes = [P, C.c_int64, I64P, F32P]
        L.mlp_profile_set.argtypes = [P, C.c_int, C.c_int, F32P]
        if hasattr(L, 'mlp_pool_info'):   # (experiment builds of older sources lack it)
            L.mlp_pool_info.argtypes = [C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
            L.mlp_pool_trim.argtypes = [C.c_int]
        _LIB = L
    return _LIB


EXPORTED = ['mlp_ctx_create', 'mlp_ctx_destroy', 'mlp_last_error', 'mlp_set_scratch', 'mlp_family_load',
            'mlp_family_npairs', 'mlp_posteriors', 'mlp_pair_results', 'mlp_csr_total',
            'mlp_csr_export', 'mlp_csr_import', 'mlp_relax', 'mlp_relax_qp',
            'mlp_relax_qp_selective', 'mlp_profile_posterior', 'mlp_profile_posterior_cpnp', 'mlp_profile_result', 'mlp_viterbi', 'mlp_viterbi_results',
            'mlp_viterbi_path', 'mlp_model_adjustment', 'mlp_family_features', 'mlp_comm_unique_id', 'mlp_comm_init',
            'mlp_shard_range', 'mlp_shard_plan', 'mlp_gather_layout', 'mlp_allgather', 'mlp_synchronize', 'mlp_profile',
            'mlp_kernel_times', 'mlp_profile_reset', 'mlp_ctx_create_mask', 'mlp_set_shards', 'mlp_shard_count',
            'mlp_relax_shard_plan', 'mlp_ctx_create_host', 'mlp_ctx_is_host', 'mlp_relax_blockmfma_eval',
            'mlp_profile_defer', 'mlp_profile_mea', 'mlp_profile_gather', 'mlp_relax_range', 'mlp_profile_set',
            'mlp_pool_info', 'mlp_pool_trim']


def pool_info(device=0):
    """(held, free) bytes of the process's device memory pool (mlp_pool_info)."""
    h, f = C.c_uint64(), C.c_uint64()
    lib().mlp_pool_info(int(device), C.byref(h), C.byref(f))
    return h.value, f.value


def pool_trim(device=0):
    """Blocks of the pool with nothing in use back to the driver (mlp_pool_trim)."""
    lib().mlp_pool_trim(int(device))


def shard_plan(lens, nranks, rank):
    """Contiguous, cell-balanced pair range [p0, p1) of `rank` (host only:
    the split mlp_shard_range applies on the GPU path)."""
    lens = np.ascontiguousarray(lens, np.int32)
    b, e = I64(), I64()
    rc = lib().mlp_shard_plan(len(lens), lens, int(nranks), int(rank), C.byref(b), C.byref(e))
    if rc != 0:
        raise MlpError(rc, 'mlp_shard_plan')
    return b.value, e.value


def relax_shard_plan(lens, pair_nnz, nranks):
    """bounds[nranks + 1] of the consistency-round output-pair ranges,
    balanced by estimated multiply-adds (host only: the split every rank and
    every in-process shard applies)."""
    lens = np.ascontiguousarray(lens, np.int32)
    nnz = np.ascontiguousarray(pair_nnz, np.int64)
    b = np.zeros(int(nranks) + 1, np.int64)
    rc = lib().mlp_relax_shard_plan(len(lens), lens, nnz, int(nranks), b)
    if rc != 0:
        raise MlpError(rc, 'mlp_relax_shard_plan')
    return b


def gather_layout(npairs, shards):
    """shards: [(p0, p1, entries)] per rank.  Returns ebase[nranks + 1], the
    global first entry of every rank's block (as mlp_allgather places them);
    raises if the ranges do not tile [0, npairs) in rank order."""
    info = np.ascontiguousarray(np.array(shards, np.int64).reshape(-1))
    eb = np.zeros(len(shards) + 1, np.int64)
    rc = lib().mlp_gather_layout(len(shards), int(npairs), info, eb)
    if rc != 0:
        raise MlpError(rc, 'shards must tile the pair range in rank order')
    return eb


def pair_index(n, a, b):
    """Row-major index of pair (a, b), a < b (CPNP/MSA.cpp:907-919)."""
    return a * n - a * (a + 1) // 2 + (b - a - 1)


def pairs_of(n):
    return [(a, b) for a in range(n) for b in range(a + 1, n)]


class Family:
    """One MLProbs family resident on one GPU."""

    def __init__(self, seqs, device=0, device_mask=None, shards=None, host=False):
        """device: one GPU; device_mask: every GPU of the mask from this one
        context (mlp_ctx_create_mask); shards: force that many shards (virtual
        shards may share a GPU); host: the host-CPU context
        (mlp_ctx_create_host), no GPU involved."""
        self._L = lib()
        self._ctx = C.c_void_p()
        if host:
            self._chk(self._L.mlp_ctx_create_host(C.byref(self._ctx)), ctx=False)
        elif device_mask is not None or shards:
            mask = device_mask if device_mask is not None else (1 << int(device))
            self._chk(self._L.mlp_ctx_create_mask(int(mask), C.byref(self._ctx)), ctx=False)
        else:
            self._chk(self._L.mlp_ctx_create(int(device), C.byref(self._ctx)), ctx=False)
        if shards:
            self._chk(self._L.mlp_set_shards(self._ctx, int(shards)), ctx=False)
        self.seqs = [s.upper() for s in seqs]
        self.n = len(self.seqs)
        self.lens = np.array([len(s) for s in self.seqs], np.int64)
        offs = np.zeros(self.n + 1, np.int64)
        offs[1:] = np.cumsum(self.lens)
        self._chk(self._L.mlp_family_load(self._ctx, self.n, ''.join(self.seqs).encode(), offs))
        self.npairs = self.n * (self.n - 1) // 2
        rp = np.zeros(self.npairs + 1, np.int64)
        k = 0
        for a in range(self.n):
            for b in range(a + 1, self.n):
                rp[k + 1] = rp[k] + self.lens[a] + 2
                k += 1
        self.rp_off = rp
        self._csr = None

    def set_scratch(self, nbytes):
        """Device bytes the posterior stage may hold as batch scratch
        (mlp_set_scratch; small budgets mean several batches and the PF
        posterior in the Zm slots)."""
        self._chk(self._L.mlp_set_scratch(self._ctx, int(nbytes)))

    def _chk(self, rc, ctx=True):
        if rc != 0:
            msg = self._L.mlp_last_error(self._ctx).decode() if ctx else 'context creation failed'
            raise MlpError(rc, msg)

    def close(self):
        if self._ctx:
            self._L.mlp_ctx_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- posterior stage
    def posteriors(self, pid, delta, p_begin=0, p_end=None):
        p_end = self.npairs if p_end is None else p_end
        self._csr = None
        self._chk(self._L.mlp_posteriors(self._ctx, int(pid), float(delta), int(p_begin), int(p_end)))

    def results(self, p_begin=0, p_end=None):
        p_end = self.npairs if p_end is None else p_end
        m = p_end - p_begin
        d = np.zeros(m, np.float32)
        e = np.zeros(m, np.float32)
        z = np.zeros(m, np.int64)
        self._chk(self._L.mlp_pair_results(self._ctx, p_begin, p_end, d.ctypes.data, e.ctypes.data, z.ctypes.data))
        return d, e, z

    def distances(self):
        d, _, _ = self.results()
        D = np.zeros((self.n, self.n), np.float32)
        k = 0
        for a in range(self.n):
            for b in range(a + 1, self.n):
                D[a, b] = D[b, a] = d[k]
                k += 1
        return D

    def export(self):
        tot = I64(0)
        self._chk(self._L.mlp_csr_total(self._ctx, C.byref(tot)))
        rp = np.zeros(int(self.rp_off[-1]), np.int32)
        eo = np.zeros(self.npairs + 1, np.int64)
        cols = np.zeros(max(tot.value, 1), np.uint16)
        vals = np.zeros(max(tot.value, 1), np.float32)
        self._chk(self._L.mlp_csr_export(self._ctx, rp.ctypes.data, eo.ctypes.data, cols.ctypes.data, vals.ctypes.data))
        self._csr = (rp, eo, cols[:tot.value], vals[:tot.value])
        return self._csr

    def import_csr(self, rp, eo, cols, vals):
        self._csr = None
        self._chk(self._L.mlp_csr_import(self._ctx, np.ascontiguousarray(rp, np.int32),
                                         np.ascontiguousarray(eo, np.int64),
                                         np.ascontiguousarray(cols, np.uint16),
                                         np.ascontiguousarray(vals, np.float32)))

    def sparse(self, p):
        """(row_ptr[L_a+2], cols, vals) of pair index p (SparseMatrix layout)."""
        if self._csr is None:
            self.export()
        rp, eo, cols, vals = self._csr
        r = rp[self.rp_off[p]:self.rp_off[p + 1]]
        e0, e1 = eo[p], eo[p + 1]
        return r, cols[e0:e1].astype(np.int32), vals[e0:e1]

    # ---- consistency
    def relax_qp(self, iters, weights, sel_dist=None, selectivity=200.0):
        """QuickProbs' consistency rounds (include/mlpgpu.h mlp_relax_qp,
        mlp_relax_qp_selective with an N x N selectivity distance matrix)."""
        w = np.ascontiguousarray(weights, np.float32)
        assert len(w) == self.n
        self._csr = None
        if sel_dist is None:
            self._chk(self._L.mlp_relax_qp(self._ctx, int(iters), w))
            return
        d = np.ascontiguousarray(sel_dist, np.float32)
        assert d.shape == (self.n, self.n)
        self._chk(self._L.mlp_relax_qp_selective(self._ctx, int(iters), w, d.ctypes.data, float(selectivity)))

    def profile_posterior(self, weights, labels1, maps1, L1, labels2, maps2, L2):
        """Weighted profile-profile posterior (include/mlpgpu.h
        mlp_profile_posterior); maps: per sequence its getMapping array."""
        w = np.ascontiguousarray(weights, np.float32)
        l1 = np.ascontiguousarray(labels1, np.int32)
        l2 = np.ascontiguousarray(labels2, np.int32)
        m1 = np.ascontiguousarray(np.concatenate(maps1), np.int32)
        m2 = np.ascontiguousarray(np.concatenate(maps2), np.int32)
        out = np.empty((L1 + 1) * (L2 + 1), np.float32)
        self._chk(self._L.mlp_profile_posterior(self._ctx, w, len(l1), l1, int(L1), m1, len(l2), l2, int(L2), m2,
                                                out))
        return out.reshape(L1 + 1, L2 + 1)

    def profile_defer(self, on):
        """Leave the next profile posteriors on the device (mlp_profile_defer)."""
        self._chk(self._L.mlp_profile_defer(self._ctx, int(bool(on))))

    def profile_mea(self, L1, L2):
        """MEA path ('B'/'X'/'Y') and score of the last profile posterior,
        on the device (mlp_profile_mea)."""
        buf = C.create_string_buffer(L1 + L2 + 1)
        n = C.c_int32(0)
        sc = C.c_float(0)
        self._chk(self._L.mlp_profile_mea(self._ctx, buf, C.byref(n), C.byref(sc)))
        return buf.raw[:n.value].decode(), np.float32(sc.value)

    def profile_set(self, post):
        """Make a host (L1 + 1) x (L2 + 1) posterior the device-resident
        matrix for profile_mea / profile_gather (mlp_profile_set)."""
        p = np.ascontiguousarray(post, np.float32)
        self._chk(self._L.mlp_profile_set(self._ctx, p.shape[0] - 1, p.shape[1] - 1, p.reshape(-1)))

    def profile_gather(self, cells):
        c = np.ascontiguousarray(cells, np.int64)
        out = np.empty(len(c), np.float32)
        self._chk(self._L.mlp_profile_gather(self._ctx, len(c), c, out))
        return out

    def relax_blockmfma_eval(self, xs, ys):
        """Dense-block MFMA evaluation of one consistency round's transform
        (include/mlpgpu.h mlp_relax_blockmfma_eval); returns a dict."""
        x = np.ascontiguousarray(xs, np.int32)
        y = np.ascontiguousarray(ys, np.int32)
        res = np.zeros(7, np.float64)
        self._chk(self._L.mlp_relax_blockmfma_eval(self._ctx, len(x), x, len(y), y, res.ctypes.data))
        keys = ('seconds', 'dense_macs', 'outputs', 'max_rel_err', 'cells_checked', 'tiles', 'blocks')
        return {k: float(v) for k, v in zip(keys, res)}

    def relax(self, iters):
        self._csr = None
        self._chk(self._L.mlp_relax(self._ctx, int(iters)))

    def relax_range(self, r0, r1):
        """One C_P_NP_Aln round over output pairs [r0, r1) (one rank's share,
        mlp_relax_range); the store then holds that block, entries from 0."""
        self._csr = None
        self._chk(self._L.mlp_relax_range(self._ctx, int(r0), int(r1)))

    # ---- multi-GPU
    @staticmethod
    def unique_id():
        buf = C.create_string_buffer(128)
        rc = lib().mlp_comm_unique_id(buf)
        if rc:
            raise MlpError(rc, 'ncclGetUniqueId')
        return buf.raw

    def comm_init(self, uid, nranks, rank):
        self._chk(self._L.mlp_comm_init(self._ctx, uid, int(nranks), int(rank)))

    def shard(self, nranks, rank):
        b, e = I64(0), I64(0)
        self._chk(self._L.mlp_shard_range(self._ctx, nranks, rank, C.byref(b), C.byref(e)))
        return b.value, e.value

    def allgather(self):
        self._csr = None
        self._chk(self._L.mlp_allgather(self._ctx))

    def synchronize(self):
        self._chk(self._L.mlp_synchronize(self._ctx))

    # ---- profiling
    def profile(self, enable=True):
        self._chk(self._L.mlp_profile(self._ctx, 1 if enable else 0))
        self._chk(self._L.mlp_profile_reset(self._ctx))

    # ---- family test (CPNP/MSA.cpp:646-882)
    def viterbi(self, keep_paths=False, p_begin=0, p_end=None):
        """Viterbi alignment of pairs [p_begin, p_end) (ComputeViterbiAlignment,
        CPNP/ProbabilisticModel.h:1043-1170)."""
        p_end = self.npairs if p_end is None else p_end
        self._chk(self._L.mlp_viterbi(self._ctx, int(p_begin), int(p_end), int(bool(keep_paths))))

    def viterbi_results(self):
        """(identical residues in match columns, path length) per pair."""
        m = np.zeros(self.npairs, np.float32)
        n = np.zeros(self.npairs, np.int32)
        self._chk(self._L.mlp_viterbi_results(self._ctx, 0, self.npairs, m.ctypes.data, n.ctypes.data))
        return m, n

    def viterbi_path(self, p):
        """Path of pair p as the reference's string of 'B' / 'X' / 'Y'."""
        a, b = pairs_of(self.n)[p]
        buf = np.zeros(self.lens[a] + self.lens[b], np.uint8)
        n = C.c_int32()
        self._chk(self._L.mlp_viterbi_path(self._ctx, int(p), buf.ctypes.data, C.byref(n)))
        return ''.join('BXY'[x] for x in buf[: n.value])

    def model_adjustment(self):
        """ModelAdjustmentTest (CPNP/MSA.cpp:775-882): (identity, variance,
        delta, code) with code = variance_mean + identity class."""
        idn, var, dl = C.c_float(), C.c_float(), C.c_float()
        code = C.c_int32()
        self._chk(self._L.mlp_model_adjustment(self._ctx, C.byref(idn), C.byref(var), C.byref(dl), C.byref(code)))
        return idn.value, var.value, dl.value, code.value

    def family_features(self, theta=1.0):
        """Alter_ModelAdjustmentTest (CPNP/MSA.cpp:646-772), the `-G` line:
        (identity, variance, N, avg_len, tmp_sp, peak_ratio, factor)."""
        f = np.zeros(5, np.float32)
        ints = np.zeros(2, np.int32)
        self._chk(self._L.mlp_family_features(self._ctx, C.c_float(theta), f.ctypes.data, ints.ctypes.data))
        return (float(f[0]), float(f[1]), int(ints[0]), int(ints[1]), float(f[2]), float(f[3]), float(f[4]))

    @staticmethod
    def features_line(feat):
        """The `-G` output line (std::to_string of each field, tab-separated,
        CPNP/MSA.cpp:771)."""
        i, v, n, al, sp, pk, fa = feat
        return '\t'.join(['%f' % i, '%f' % v, str(n), str(al), '%f' % sp, '%f' % pk, '%f' % fa])

    def kernel_times(self):
        ms = np.zeros(len(KERNELS), np.float64)
        nl = np.zeros(len(KERNELS), np.int64)
        cells = np.zeros(len(KERNELS), np.int64)
        self._chk(self._L.mlp_kernel_times(self._ctx, ms.ctypes.data, nl.ctypes.data, cells.ctypes.data))
        return {k: {'ms': float(ms[i]), 'launches': int(nl[i]), 'cells': int(cells[i])}
                for i, k in enumerate(KERNELS)}
