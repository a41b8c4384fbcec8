"""bench.py -- all-pairs posterior stage of C_P_NP_Aln on MI355X.

One step = the whole posterior stage over the family:
every pair's 5-state + partition-function + local posteriors, RMS merge,
MEA distance and sparsification into the canonical CSR store, inputs already
resident in HBM.  With N GPUs the pairs are split into N contiguous,
cell-balanced shards (one process per GPU) and the step ends with the RCCL
all-gather of the sparse posteriors over xGMI (the exchange step before
consistency).  Value = pair-cells of the whole family / max-over-ranks time.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 512] [--len 400]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = 'pair-HMM DP cell updates/s (all-pairs) + end-to-end MSA sec/family'
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# VALU issue peak: 256 CUs x 4 SIMD-32 x 2.4 GHz, one wave64 VALU instruction
# per 2 cycles per SIMD (MI355X_MICROARCH.md, "Wave scheduling").  Measured
# (tools/probe/valu_rate, profiles/r05c_valu_rate_operands.json): v_add / mul /
# fma_f32, v_add_u32, v_and, v_bitop3 with VGPR, literal or inline operands at
# 2.3-2.5 cycles (1.0-1.1e12 wave-instr/s at 8 waves per SIMD); any VALU
# instruction with an SGPR operand, v_max / min_f32, v_cvt_i32_f32, v_bcnt,
# v_lshl_add, v_mov_dpp, f64 and packed f32 at 4.3-4.5 cycles (half this peak)
VALU_PEAK_WAVE_INSTS = 256 * 4 * 2.4e9 / 2
# Algorithmic HBM bytes per pair-cell for each kernel of the pid-0 pipeline
# ("Kernels and their rooflines"), round-3 layout: the forward
# writes f5, local f and PF Zm (4 + 4 + 8); the backward reads f5 and Zm and
# writes f5 (f + b), local b and the PF posterior (12 + 12); the local totals
# stream local f (4); the merge reads f5, local f, local b, PF posterior (16).
ALGO_BYTES = {'forward': 16, 'backward': 24, 'local_totals': 4, 'merge_mea_sparsify': 16}
STAGE_BYTES = 56  # pid 0/1 algorithmic bytes per pair-cell
# mlprobs --trace stages in pipeline order (tools/c5_attribution.py) and the
# committed per-family cause of every C5 family whose output differs from the
# reference CLIs' multi-threaded runs
C5_STAGES = ('features_line', 'class1', 'col_score', 'regions', 'realigned', 'output')
C5_ATTRIBUTION = 'r05_c5_attribution_recheck.json'
# the clock every C5 run reads (the -p 1 refinement's srand(time(0)), CPNP/MSA.cpp:1896)
C5_CLOCK = '1700000000'
# the printed line stays far below what the driver parses (round 5's 20 KB
# line was not parsed); the full record goes to DETAIL_PATH
LINE_LIMIT = 8000
DETAIL_PATH = os.environ.get('MLP_BENCH_DETAIL', os.path.join(ROOT, 'gpurun_out', 'bench_detail.json'))


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--n', '--nseq', dest='n', type=int, default=512)  # (--nseq: under torchrun, --n is ambiguous)
    ap.add_argument('--len', type=int, default=400)
    ap.add_argument('--s', type=float, default=0.7)
    ap.add_argument('--seed', type=int, default=11)
    ap.add_argument('--pid', type=int, default=0)
    ap.add_argument('--delta', type=float, default=0.132548)
    ap.add_argument('--cpu-pairs', type=int, default=6144, help='reference CPU baseline sample (pairs)')
    ap.add_argument('--cpu-threads', type=int, default=16)
    ap.add_argument('--no-cpu', action='store_true')
    ap.add_argument('--relax', type=int, default=-1,
                    help='also time N consistency rounds (C4; reported separately; default 4 on one GPU, 0 on several)')
    ap.add_argument('--relax-cpu-pairs', type=int, default=768, help='reference DoRelaxation sample (output pairs)')
    ap.add_argument('--no-e2e', action='store_true',
                    help='skip the end-to-end c_p_np_aln / quickprobs family timings')
    ap.add_argument('--no-qp', action='store_true', help='skip the QuickProbs posterior/consistency timings')
    ap.add_argument('--e2e-runs', type=int, default=3, help='fresh-process runs per end-to-end leg')
    ap.add_argument('--no-shards', action='store_true', help='skip the 8-virtual-shard all-gather timing')
    ap.add_argument('--c5-stride', type=int, default=1,
                    help='C5 leg over every k-th TEST/ox + sabre family (default 1: all 818)')
    ap.add_argument('--no-c5', action='store_true', help='skip the C5 pipeline leg')
    ap.add_argument('--c5-ref', choices=('all', 'sample', 'none'), default='sample',
                    help='reference-CLI leg of C5: every family (minutes), a sample (every 8th family plus the '
                         'heavy golden families; default) or none')
    ap.add_argument('--only-c5', action='store_true', help='run the C5 leg only and print its JSON')
    ap.add_argument('--host', action='store_true',
                    help='N ranks on host contexts over gloo: the CPU dry run of the multi-rank path '
                         '(tests/test_multirank_cpu.py); no GPU')
    return ap.parse_args()


def log(msg):
    """Progress on stderr (a long silent run looks hung to the GPU box's watchdog)."""
    print(f'[bench {time.strftime("%H:%M:%S")}] {msg}', file=sys.stderr, flush=True)


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import orc
    return orc


def read_pair_dump(path):
    """oracle/ref_probe's per-pair dump (dump_pairs): pair ids, L1, distances,
    MEA scores and the sparse rows in the canonical layout."""
    with open(path, 'rb') as fh:
        buf = fh.read()
    npairs = int(np.frombuffer(buf, np.int64, 1, 0)[0])
    off = 8
    ab, L1, dist, mea, rps, cols, vals, eo = [], [], [], [], [], [], [], [0]
    for _ in range(npairs):
        a, b, la = (int(x) for x in np.frombuffer(buf, np.int32, 3, off))
        d, m = np.frombuffer(buf, np.float32, 2, off + 12)
        nnz = int(np.frombuffer(buf, np.int64, 1, off + 20)[0])
        off += 28
        rps.append(np.frombuffer(buf, np.int32, la + 2, off))
        off += 4 * (la + 2)
        cols.append(np.frombuffer(buf, np.int32, nnz, off))
        off += 4 * nnz
        vals.append(np.frombuffer(buf, np.float32, nnz, off))
        off += 4 * nnz
        ab.append((a, b))
        L1.append(la)
        dist.append(d)
        mea.append(m)
        eo.append(eo[-1] + nnz)
    L1 = np.array(L1, np.int32)
    return {'ab': ab, 'L1': L1, 'dist': np.array(dist, np.float32), 'mea': np.array(mea, np.float32),
            'roff': np.concatenate([[0], np.cumsum(L1.astype(np.int64) + 2)[:-1]]).astype(np.int64),
            'eoff': np.array(eo[:-1], np.int64), 'rp': np.concatenate(rps).astype(np.int32),
            'cols': np.concatenate(cols + [np.zeros(1, np.int32)]).astype(np.int32),
            'vals': np.concatenate(vals + [np.zeros(1, np.float32)]).astype(np.float32)}


def compare_with_dump(orc, dump, n, lens, store, exact):
    """Parity readouts: the reference's sparse rows of
    the dumped pairs against the GPU store (section 8c rule)."""
    pairs = np.array([orc.pair_index(n, a, b) for a, b in dump['ab']], np.int64)
    g_rp, g_eo, g_cols, g_vals = store
    L1, ro, eo = orc.store_view(lens, pairs, g_rp, g_eo)
    st = orc.csr_compare(dump['L1'], (dump['roff'], dump['eoff'], dump['rp'], dump['cols'], dump['vals']),
                         (ro, eo, g_rp, g_cols, g_vals))
    st['symmetric_difference'] = st.pop('cutoff_flips')
    if exact:
        st['bit_exact'] = st['inexact'] == 0
    return pairs, st


def cpu_baseline(fasta, args, n, lens, store, gpu_dist):
    """The reference's own pair loop (oracle/_ref/ref_probe, compiled from
    /root/reference by `make -C oracle ref`) timed on a bounded sample of the
    same family, and its output for that sample compared with the GPU store
    (same-run parity readouts); the plain-C port when the reference build is
    absent (timing only)."""
    probe = os.path.join(ROOT, 'oracle', '_ref', 'ref_probe')
    orc = _oracle()
    if os.path.exists(probe):
        with tempfile.TemporaryDirectory() as td:
            dump = os.path.join(td, 'ref.bin')
            out = subprocess.run([probe, 'bench', fasta, str(args.pid), str(args.cpu_pairs), str(args.cpu_threads),
                                  dump], capture_output=True, text=True, timeout=900,
                                 env=dict(os.environ, REF_PROBE_DELTA=repr(args.delta)))
            if out.returncode == 0:
                r = json.loads(out.stdout.strip().splitlines()[-1])
                res = {'value': r['pair_cells_per_s'], 'unit': 'pair-cells/s', 'cores': args.cpu_threads,
                       'kind': 'reference',
                       'sample': f"first {r['pairs']} pairs of the same family, {r['seconds']:.1f} s, "
                                 f"reference C_P_NP_Aln pdoAlign pair body (posterior+MEA+sparsify)"}
                parity = None
                if store is not None:
                    d = read_pair_dump(dump)
                    pairs, parity = compare_with_dump(orc, d, n, lens, store, exact=args.pid == 2)
                    rel = np.abs(gpu_dist[pairs] - d['dist']) / np.maximum(np.abs(d['dist']), 1e-6)
                    parity['distance_max_rel_err'] = float(rel.max())
                    parity['rule'] = ('|d| <= 1e-4 max(|ref|, 1e-6); one-sided entries within 1e-4 of the '
                                      '0.01 cutoff (SURVEY.md 8c)')
                    parity['sample'] = f'the {len(pairs)} pairs of the CPU baseline, reference output'
                return res, parity
    seqs = [s for _, s in __import__('mlprobs_amd.synth', fromlist=['x']).read_fasta(fasta)]
    m = orc.model(args.delta)
    t0 = time.perf_counter()
    orc.pair_loop(m, seqs, args.pid, max_pairs=args.cpu_pairs, threads=args.cpu_threads)
    dt = time.perf_counter() - t0
    cells = sum((len(seqs[a]) + 1) * (len(seqs[b]) + 1) for a, b in
                [(a, b) for a in range(len(seqs)) for b in range(a + 1, len(seqs))][:args.cpu_pairs])
    return {'value': cells / dt, 'unit': 'pair-cells/s', 'cores': args.cpu_threads, 'kind': 'port',
            'sample': f'first {args.cpu_pairs} pairs, {dt:.1f} s, oracle port'}, None


def store_hash(fam, results=True):
    """sha256 over the canonical store and the per-pair results (distances,
    MEA scores, entry counts): the bit-identity check between the unsharded
    and the virtually sharded runs (results=False: the store alone, which is
    what the host dry run's gloo exchange carries)."""
    import hashlib
    h = hashlib.sha256()
    for a in list(fam.export()) + (list(fam.results()) if results else []):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


class RankExchange:
    """The exchange steps of the N-rank run.  On GPUs the library's own: the
    RCCL all-gather of the posterior store (mlp_allgather) and mlp_relax,
    which relaxes this rank's MAC-balanced output range and all-gathers after
    the round, both timed by the library's kernel timers ('allgather').  With
    --host (the CPU dry run) the same placement over gloo: each rank's CSR
    block goes where mlp_gather_layout puts it and the gathered store is
    imported back (mlp_csr_import), timed on the host clock -- what
    tests/test_multirank_cpu.py checks against the single-process store."""

    def __init__(self, fam, world, rank, dist, host):
        self.fam, self.world, self.rank, self.dist, self.host = fam, world, rank, dist, host
        self.host_gather_s = 0.0
        self.received_bytes = 0

    def _place(self, r0, r1):
        from mlprobs_amd import engine
        f = self.fam
        rp_full, eo, cols, vals = f.export()
        rp = rp_full[f.rp_off[r0]:f.rp_off[r1]].astype(np.int32)
        blk = (rp, cols[int(eo[r0]):int(eo[r1])].copy(), vals[int(eo[r0]):int(eo[r1])].copy())
        shards = [None] * self.world
        self.dist.all_gather_object(shards, (r0, r1, int(len(blk[1]))))
        ebase = engine.gather_layout(f.npairs, shards)
        blocks = [None] * self.world
        self.dist.all_gather_object(blocks, blk)
        g_rp = np.concatenate([b[0] for b in blocks])
        g_cols = np.zeros(int(ebase[-1]), np.uint16)
        g_vals = np.zeros(int(ebase[-1]), np.float32)
        for r, b in enumerate(blocks):
            g_cols[ebase[r]:ebase[r + 1]] = b[1]
            g_vals[ebase[r]:ebase[r + 1]] = b[2]
        g_eo = np.zeros(f.npairs + 1, np.int64)
        g_eo[1:] = np.cumsum(g_rp[np.asarray(f.rp_off[1:], np.int64) - 1])
        f.import_csr(g_rp, g_eo, g_cols, g_vals)

    def gather(self, p0, p1):
        """After this rank's posterior range: every rank's block everywhere."""
        if not self.host:
            self.fam.allgather()
            return
        t0 = time.perf_counter()
        self._place(p0, p1)
        self.host_gather_s += time.perf_counter() - t0

    def relax_round(self, lens):
        """One consistency round over this rank's output range, then the gather."""
        if not self.host:
            self.fam.relax(1)
            return
        from mlprobs_amd import engine
        _, eo, _, _ = self.fam.export()
        bounds = engine.relax_shard_plan(np.asarray(lens, np.int32), np.diff(eo), self.world)
        r0, r1 = int(bounds[self.rank]), int(bounds[self.rank + 1])
        self.fam.relax_range(r0, r1)
        t0 = time.perf_counter()
        self._place(r0, r1)
        self.host_gather_s += time.perf_counter() - t0

    def gather_ms(self, kt):
        return self.host_gather_s * 1e3 if self.host else kt['allgather']['ms']

    def reset(self):
        self.host_gather_s = 0.0


def gather_bytes_of(fam, p0=0, p1=None):
    """Bytes of the canonical store of pairs [p0, p1): entries (uint16 column
    + fp32 value), row pointers (int32) and per-pair results (distance, MEA
    score, entry count: 16 B) -- what the all-gather moves."""
    p1 = fam.npairs if p1 is None else p1
    nnz = fam.results()[2]
    return (int(nnz[p0:p1].sum()) * 6 + int(fam.rp_off[p1] - fam.rp_off[p0]) * 4 + (p1 - p0) * 16)


def group_roofline(kt, steps):
    """The dominant kernel group of this rank's posterior stage and its HBM
    roofline (algorithmic bytes per launch / average launch time)."""
    cand = [k for k in ALGO_BYTES if kt[k]['launches']]
    if not cand:
        return None
    dom = max(cand, key=lambda k: kt[k]['ms'])
    launches = max(kt[dom]['launches'], 1)
    avg_ms = kt[dom]['ms'] / launches
    achieved = ALGO_BYTES[dom] * kt[dom]['cells'] / launches / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    return {'bound': 'hbm', 'kernel': dom, 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': achieved / HBM_PEAK_GBS, 'avg_launch_ms': avg_ms, 'algo_bytes_per_cell': ALGO_BYTES[dom]}


def multirank_legs(fam, ex, args, world, rank, dist, lens, p0, p1, dt, kt, sync):
    """Per-rank records of the N-rank run (rank 0 gets the list): pairs,
    pair-cells, posterior and all-gather time per step, the bytes the gather
    brought in and its rate, the rank's dominant kernel roofline; then
    args.relax consistency rounds, each timed as the max over ranks with its
    per-rank relaxation-kernel and gather times."""
    gms = ex.gather_ms(kt) / args.steps
    recv = gather_bytes_of(fam) - gather_bytes_of(fam, p0, p1)
    cells = int(sum((lens[a] + 1) * (lens[b] + 1) for a, b in
                    __import__('mlprobs_amd.engine', fromlist=['x']).pairs_of(len(lens))[p0:p1]))
    me = {'rank': rank, 'pairs': p1 - p0, 'pair_cells': cells,
          'step_ms': dt / args.steps * 1e3, 'gather_ms': gms,
          'posterior_ms': dt / args.steps * 1e3 - gms, 'gather_bytes_in': recv,
          'gather_GBps': recv / (gms * 1e-3) / 1e9 if gms > 0 else None,
          'kernels_ms_per_step': {k: v['ms'] / args.steps for k, v in kt.items() if v['launches']},
          'roofline': group_roofline(kt, args.steps),
          'store_hash': store_hash(fam, results=False)}  # every rank must hold the same gathered store
    ranks = [None] * world
    dist.all_gather_object(ranks, me)
    relax = None
    if args.relax > 0:
        per = []
        for _ in range(args.relax):
            fam.profile(True)
            ex.reset()
            sync()
            t0 = time.perf_counter()
            ex.relax_round(lens)
            sync()
            rdt = time.perf_counter() - t0
            kr = fam.kernel_times()
            mine = {'rank': rank, 'seconds': rdt, 'relax_kernel_ms': kr['relax']['ms'], 'gather_ms': ex.gather_ms(kr),
                    'store_hash': store_hash(fam, results=False)}
            allr = [None] * world
            dist.all_gather_object(allr, mine)
            per.append({'seconds': max(r['seconds'] for r in allr), 'gather_ms': max(r['gather_ms'] for r in allr),
                        'nnz_out': int(fam.results()[2].sum()), 'ranks': allr})
        relax = {'rounds': len(per), 'per_round': per, 'seconds': sum(r['seconds'] for r in per)}
    return ranks, relax


def relax_work(n, lens, store):
    """The reference's multiply-adds for one consistency round over this store
    (for output (x, y) and each z, every entry of P_xz meets
    the row of P_zy it selects), without enumerating them: with V_z[s][k] the
    number of entries of block {s, z} at residue k of z, MACs(x, y) =
    sum_z <V_z[x], V_z[y]>.  Returns (V, total MACs)."""
    rp, eo, cols, _ = store
    lens = np.asarray(lens, np.int64)
    K = int(lens.max()) + 1
    P = n * (n - 1) // 2
    a_of = np.repeat(np.arange(n), np.arange(n - 1, -1, -1))[:P]
    b_of = np.concatenate([np.arange(a + 1, n) for a in range(n)])
    rp_off = np.zeros(P + 1, np.int64)
    rp_off[1:] = np.cumsum(lens[a_of] + 2)
    V = np.zeros((n, n, K), np.int32)
    step = 4096
    for p0 in range(0, P, step):
        p1 = min(P, p0 + step)
        for p in range(p0, p1):  # rows of a: row lengths
            La = lens[a_of[p]]
            r = rp[rp_off[p]: rp_off[p] + La + 2]
            V[a_of[p], b_of[p], 1:La + 1] = np.diff(r[1:])
        e0, e1 = int(eo[p0]), int(eo[p1])
        pid_of = np.repeat(np.arange(p1 - p0), np.diff(eo[p0:p1 + 1]))
        cnt = np.bincount(pid_of * K + cols[e0:e1].astype(np.int64), minlength=(p1 - p0) * K).reshape(p1 - p0, K)
        V[b_of[p0:p1], a_of[p0:p1], :] = cnt  # columns of b: column counts
    total = 0
    for z in range(n):
        v = V[z].astype(np.int64)
        total += int(((v.sum(0) ** 2) - (v * v).sum(0)).sum()) // 2
    return V, total


def relax_leg(fam, args, n, lens, total_cells):
    """C4 on one GPU: `args.relax` consistency rounds (CPNP/MSA.cpp:1172-1360)
    over the posterior store, timed per round, with the section 8d accounting
    of round 1 (reference multiply-adds, algorithmic bytes 16 (N - 1) nnz,
    HBM roofline of k_relax_tile) and, on rank 0 with --cpu, the reference's
    DoRelaxation timed on a strided sample of output pairs from the same input
    and compared with the GPU's output for them."""
    store0 = [a.copy() for a in fam.export()]
    nnz0 = int(store0[1][-1])
    V, macs = relax_work(n, lens, store0)
    rounds = []
    store1 = None
    for it in range(args.relax):
        fam.profile(True)
        fam.synchronize()
        t0 = time.perf_counter()
        fam.relax(1)
        fam.synchronize()
        dt = time.perf_counter() - t0
        kt = fam.kernel_times()
        nnz = int(fam.results()[2].sum())
        rounds.append({'seconds': dt, 'nnz_in': nnz0 if it == 0 else rounds[-1]['nnz_out'], 'nnz_out': nnz,
                       'kernels_ms': {k: v['ms'] for k, v in kt.items() if v['launches']}})
        if it == 0:
            hash1 = store_hash(fam)
            k_ms = kt['relax']['ms'] or dt * 1e3  # host contexts (--host) time no kernels
            k_launch = max(kt['relax']['launches'], 1)
            if not args.no_cpu:
                store1 = [a.copy() for a in fam.export()]
    algo = 16.0 * (n - 1) * nnz0
    traffic = None
    pmc = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')
    if os.path.exists(pmc):
        with open(pmc) as fh:
            g = json.load(fh).get('relax')
        if g:
            traffic = g['traffic_bytes_per_nnz_in'] * nnz0 / k_launch / 1e9
    res = {'rounds': len(rounds), 'per_round': rounds, 'seconds': sum(r['seconds'] for r in rounds),
           'round1_hash': hash1,
           'nnz_per_round': [nnz0] + [r['nnz_out'] for r in rounds],
           'round1': {'macs_reference': macs, 'mac_per_s': macs / (k_ms * 1e-3), 'flop_per_s': 2 * macs / (k_ms * 1e-3),
                      'kernel_ms': k_ms},
           'roofline': {'bound': 'hbm', 'kernel': 'k_relax_tile', 'achieved': algo / k_launch / (k_ms / k_launch * 1e-3) / 1e9,
                        'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                        'frac': algo / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 'traffic': traffic,
                        'algo_bytes': algo, 'algo_rule': '16 (N - 1) nnz_in (SURVEY.md 8d: every operand block '
                                                         'read once per output pair, output read + written once)',
                        'avg_launch_ms': k_ms / k_launch}}
    probe = os.path.join(ROOT, 'oracle', '_ref', 'ref_probe')
    if store1 is not None and os.path.exists(probe):
        orc = _oracle()
        from mlprobs_amd import synth
        with tempfile.TemporaryDirectory() as td:
            fa = os.path.join(td, 'fam.fa')
            synth.write_fasta(fa, [('s%04d' % k, s) for k, s in enumerate(fam.seqs)])
            path = os.path.join(td, 'store.bin')
            rp, eo, cols, vals = store0
            with open(path, 'wb') as fh:
                fh.write(np.array([len(eo) - 1, int(eo[-1])], np.int64).tobytes())
                fh.write(rp.tobytes())
                fh.write(eo.tobytes())
                fh.write(cols.tobytes())
                fh.write(vals.tobytes())
            dump = os.path.join(td, 'relax.bin')
            out = subprocess.run([probe, 'relaxbench', fa, path, str(args.relax_cpu_pairs), str(args.cpu_threads),
                                  dump], capture_output=True, text=True, timeout=900)
            if out.returncode == 0:
                r = json.loads(out.stdout.strip().splitlines()[-1])
                d = read_pair_dump(dump)
                pairs, st = compare_with_dump(orc, d, n, lens, store1, exact=True)
                sample_macs = 0
                for a, b in d['ab']:
                    sample_macs += int(np.einsum('zk,zk->', V[:, a, :].astype(np.int64), V[:, b, :].astype(np.int64)))
                res['cpu_baseline'] = {'value': sample_macs / r['seconds'], 'unit': 'MAC/s (reference multiply-adds)',
                                       'cores': args.cpu_threads, 'kind': 'reference',
                                       'sample': f"{r['pairs']} output pairs (every {r['stride']}th), "
                                                 f"{r['seconds']:.1f} s, reference MSA::DoRelaxation on the "
                                                 "GPU's posterior store"}
                res['speedup_vs_cpu'] = res['round1']['mac_per_s'] / res['cpu_baseline']['value']
                st['sample'] = 'the CPU baseline pairs: reference DoRelaxation output vs GPU round 1'
                res['parity'] = st
            else:
                res['cpu_baseline_error'] = out.stderr[-400:]
    return res


# ---- MSA readouts: MLProbs' own SP score and TC
_ALPHA = 'ARNDCQEGHILKMFPSTWYV'
_BLOSUM62 = np.array([
    [4, -1, -2, -2, 0, -1, -1, 0, -2, -1, -1, -1, -1, -2, -1, 1, 0, -3, -2, 0],
    [-1, 5, 0, -2, -3, 1, 0, -2, 0, -3, -2, 2, -1, -3, -2, -1, -1, -3, -2, -3],
    [-2, 0, 6, 1, -3, 0, 0, 0, 1, -3, -3, 0, -2, -3, -2, 1, 0, -4, -2, -3],
    [-2, -2, 1, 6, -3, 0, 2, -1, -1, -3, -4, -1, -3, -3, -1, 0, -1, -4, -3, -3],
    [0, -3, -3, -3, 9, -3, -4, -3, -3, -1, -1, -3, -1, -2, -3, -1, -1, -2, -2, -1],
    [-1, 1, 0, 0, -3, 5, 2, -2, 0, -3, -2, 1, 0, -3, -1, 0, -1, -2, -1, -2],
    [-1, 0, 0, 2, -4, 2, 5, -2, 0, -3, -3, 1, -2, -3, -1, 0, -1, -3, -2, -2],
    [0, -2, 0, -1, -3, -2, -2, 6, -2, -4, -4, -2, -3, -3, -2, 0, -2, -2, -3, -3],
    [-2, 0, 1, -1, -3, 0, 0, -2, 8, -3, -3, -1, -2, -1, -2, -1, -2, -2, 2, -3],
    [-1, -3, -3, -3, -1, -3, -3, -4, -3, 4, 2, -3, 1, 0, -3, -2, -1, -3, -1, 3],
    [-1, -2, -3, -4, -1, -2, -3, -4, -3, 2, 4, -2, 2, 0, -3, -2, -1, -2, -1, 1],
    [-1, 2, 0, -1, -3, 1, 1, -2, -1, -3, -2, 5, -1, -3, -1, 0, -1, -3, -2, -2],
    [-1, -1, -2, -3, -1, 0, -2, -3, -2, 1, 2, -1, 5, 0, -2, -1, -1, -1, -1, 1],
    [-2, -3, -3, -3, -2, -3, -3, -3, -1, 0, 0, -3, 0, 6, -4, -2, -2, 1, 3, -1],
    [-1, -2, -2, -1, -3, -1, -1, -2, -2, -3, -3, -1, -2, -4, 7, -1, -1, -4, -3, -2],
    [1, -1, 1, 0, -1, 0, 0, 0, -1, -2, -2, 0, -1, -2, -1, 4, 1, -3, -2, -2],
    [0, -1, 0, -1, -1, -1, -1, -2, -2, -1, -1, -1, -1, -2, -1, 1, 5, -2, -2, 0],
    [-3, -3, -4, -4, -2, -2, -3, -2, -2, -3, -2, -3, -1, 1, -4, -3, -2, 11, 2, -3],
    [-2, -2, -2, -3, -2, -1, -2, -3, 2, -1, -1, -2, -1, 3, -3, -2, -2, 2, 7, -1],
    [0, -3, -3, -3, -1, -2, -2, -3, -3, 3, 1, -2, 1, -1, -2, -2, 0, -3, -1, 4]], np.int64)


def msa_rows(text):
    """Header line -> row, as MLProbs' utils parse an MSA (later duplicates win)."""
    rows, key = {}, None
    for line in text.splitlines():
        if line.startswith('>'):
            key = line
            rows[key] = ''
        elif key is not None:
            rows[key] += line.replace('\r', '')
    return rows


def sp_score(text):
    """MLProbs' un_sp (utils/calculate_column_scores.py:37-82): the mean over
    columns of the BLOSUM62 sum of pairs / (N (N - 1) / 2), gaps and
    non-standard letters scoring 0; exact integer pair sums per column."""
    rows = msa_rows(text)
    if len(rows) < 2:
        return None
    L = min(len(r) for r in rows.values())
    idx = np.full(256, 20, np.int64)
    for k, c in enumerate(_ALPHA):
        idx[ord(c)] = k
    A = np.stack([idx[np.frombuffer(r[:L].encode('latin-1'), np.uint8)] for r in rows.values()])
    cnt = np.zeros((L, 21), np.int64)
    for k in range(21):
        cnt[:, k] = (A == k).sum(0)
    c = cnt[:, :20]
    pair = np.einsum('la,ab,lb->l', c, _BLOSUM62, c) - (c * np.diag(_BLOSUM62)).sum(1)
    n = len(rows)
    col = (pair // 2) / (n * (n - 1) / 2)
    return sum(col.tolist()) / L if L else 0.0   # summed in column order, like the reference


def tc_score(text, ref_text):
    """Total-column score: the fraction of `text`'s columns that are also
    columns of `ref_text`, a column being the tuple (per shared header) of the
    residue index each row has there (-1 = gap)."""
    a, b = msa_rows(text), msa_rows(ref_text)
    keys = sorted(set(a) & set(b))
    if not keys:
        return None

    def columns(rows):
        cols = []
        mats = []
        for k in keys:
            r = np.frombuffer(rows[k].encode('latin-1'), np.uint8)
            res = (r != ord('-')) & (r != ord('.'))
            mats.append(np.where(res, np.cumsum(res) - 1, -1))
        L = min(len(m) for m in mats)
        M = np.stack([m[:L] for m in mats])
        for j in range(L):
            if (M[:, j] >= 0).any():
                cols.append(M[:, j].tobytes())
        return cols

    ca, cb = columns(a), set(columns(b))
    return sum(c in cb for c in ca) / max(len(ca), 1)


def _stages(stderr):
    st = {}
    for line in stderr.splitlines():
        if line.startswith('[stage] '):
            name, sec = line[8:].rsplit(' ', 2)[0], line.rsplit(' ', 2)[1]
            st[name] = float(sec)
    return st


def _e2e_record(runs):
    """Every run's wall time and stage split (MLP_CLI_TIMES), the median and
    the maximum; a run more than 15% above the median is named with the
    stage that grew most against the median run's split."""
    order = sorted(range(len(runs)), key=lambda k: runs[k][0])
    med_dt, r = runs[order[len(order) // 2]]
    med_st = _stages(r.stderr)
    rec = {'median_s': med_dt, 'max_s': max(x[0] for x in runs), 'runs_s': [x[0] for x in runs],
           'exit': r.returncode, 'stages_s': med_st,
           'runs': [{'s': dt, 'exit': x.returncode, 'stages_s': _stages(x.stderr)} for dt, x in runs]}
    slow = []
    for k, (dt, x) in enumerate(runs):
        if dt > 1.15 * med_dt:
            st = _stages(x.stderr)
            grew = max(st, key=lambda n: st[n] - med_st.get(n, 0.0)) if st else None
            slow.append({'run': k, 's': dt, 'stage': grew,
                         'stage_excess_s': (st[grew] - med_st.get(grew, 0.0)) if grew else None})
    rec['outliers'] = slow
    return rec, r


def _posterior_stage(rec, fam):
    """The drop-in's own posterior stage (its 16 GB scratch, a fresh process)
    beside the library headline: pair-cells per second at the median run."""
    lens = np.array([len(x) for _, x in fam], np.int64)
    cells = int(((lens + 1).sum() ** 2 - ((lens + 1) ** 2).sum()) // 2)
    post = sorted(x['stages_s'].get('posteriors', 0.0) for x in rec['runs'])
    if post and post[len(post) // 2] > 0:
        rec['posterior_stage'] = {'pair_cells': cells, 'median_s': post[len(post) // 2],
                                  'pair_cells_per_s': cells / post[len(post) // 2],
                                  'runs_s': [x['stages_s'].get('posteriors') for x in rec['runs']]}


def e2e_families(args):
    """End-to-end seconds per family of the c_p_np_aln drop-in (-p 0: family
    test, posteriors, guide tree, 2 consistency rounds, progressive alignment,
    refinement; -p 1: family test, posteriors, 2 consistency rounds, alignment
    graph, refinement), one fresh process per run (as MLProbs starts them),
    wall clock around the process; three runs each, every run listed with
    its stage split (MLP_CLI_TIMES), the median and the maximum, and any run
    more than 15% above the median named with the stage that grew.  The outputs are compared in the run with the
    reference CLI's own output on the same family where one was generated
    (tests/golden/config: -p 0 at C2 and C3, -p 1 at C2 under a fixed clock,
    MLP_SRAND_TIME), with MLProbs' SP score (un_sp) and TC against it."""
    from mlprobs_amd import synth
    cli = os.path.join(ROOT, 'mlprobs_amd', 'cli', 'c_p_np_aln')
    if not os.path.exists(cli):
        return None
    res = {}
    for tag, n, L, gold in (('C2 128x256', 128, 256, 'c2_128x256_s11'),
                            (f'C3 {args.n}x{args.len}', args.n, args.len, f'c3_{args.n}x{args.len}_s{args.seed}')):
        for mode in ('0', '1'):
            with tempfile.TemporaryDirectory() as td:
                fa = os.path.join(td, 'fam.fa')
                fam = synth.family(n, L, args.s, seed=args.seed)
                synth.write_fasta(fa, fam)
                runs = []
                # -p 1 seeds its refinement with time(0): the golden run's fixed clock
                env = dict(os.environ, MLP_CLI_TIMES='1', **({'MLP_SRAND_TIME': '1700000000'} if mode == '1' else {}))
                for _ in range(args.e2e_runs):
                    t0 = time.perf_counter()
                    r = subprocess.run([cli, '-p', mode, fa], capture_output=True, text=True, timeout=600, env=env)
                    runs.append((time.perf_counter() - t0, r))
            rec, r = _e2e_record(runs)
            _posterior_stage(rec, fam)
            log(f'e2e {tag} -p {mode}: ' + ', '.join(f'{x[0]:.2f}' for x in runs) + f' s (exit {r.returncode})')
            g = os.path.join(ROOT, 'tests', 'golden', 'config', f'{gold}.p_{mode}.out')
            if os.path.exists(g) and args.s == 0.7:
                with open(g) as fh:
                    ref = fh.read()
                rec['reference_output'] = {'identical': all(x[1].stdout == ref for x in runs),
                                           'sp_ours': sp_score(r.stdout), 'sp_reference': sp_score(ref),
                                           'tc_vs_reference': tc_score(r.stdout, ref),
                                           'reference': f'tests/golden/config/{gold}.p_{mode}.out (reference CLI, '
                                                        'single thread' + (', fixed clock)' if mode == '1' else ')')}
            res[tag if mode == '0' else f'{tag} -p 1'] = rec
    qp = os.path.join(ROOT, 'mlprobs_amd', 'cli', 'quickprobs')
    ref = os.path.join(ROOT, 'oracle', '_ref', 'quickprobs')
    if os.path.exists(qp):
        # the quickprobs drop-in (QuickProbs 2 realigner): GPU posteriors and
        # selective consistency, host tree / construction / 30-200 refinement
        # passes; at C2 also the reference QuickProbs CLI (built from its
        # sources, 16 threads) on the same input, outputs compared byte for byte
        for tag, n, L in (('quickprobs C2 128x256', 128, 256), (f'quickprobs C3 {args.n}x{args.len}', args.n, args.len)):
            with tempfile.TemporaryDirectory() as td:
                fa = os.path.join(td, 'fam.fa')
                fam = synth.family(n, L, args.s, seed=args.seed)
                synth.write_fasta(fa, fam)
                runs = []
                for _ in range(args.e2e_runs):
                    t0 = time.perf_counter()
                    r = subprocess.run([qp, fa], capture_output=True, text=True, timeout=600,
                                       env=dict(os.environ, MLP_CLI_TIMES='1'))
                    runs.append((time.perf_counter() - t0, r))
                res[tag], r = _e2e_record(runs)
                _posterior_stage(res[tag], fam)
                log(f'e2e {tag}: ' + ', '.join(f'{x[0]:.2f}' for x in runs) + f' s (exit {r.returncode})')
                g = os.path.join(ROOT, 'tests', 'golden', 'config', f'c{2 if n == 128 else 3}_{n}x{L}_s{args.seed}.qp.out')
                if os.path.exists(g) and args.s == 0.7:   # the reference QuickProbs CLI's output (gen_config_goldens.sh)
                    with open(g) as fh:
                        ref_out = fh.read()
                    res[tag]['reference_output'] = {'identical': all(x[1].stdout == ref_out for x in runs),
                                                    'reference': os.path.relpath(g, ROOT)}
                if n <= 128 and os.path.exists(ref) and not args.no_cpu:
                    t0 = time.perf_counter()
                    rr = subprocess.run([ref, '-t', str(args.cpu_threads), fa], capture_output=True, text=True,
                                        timeout=600)
                    res[tag]['reference_cpu'] = {'seconds': time.perf_counter() - t0, 'threads': args.cpu_threads,
                                                 'exit': rr.returncode, 'identical_output': rr.stdout == r.stdout}
    return res


def shard_gather(args, seqs, post_hash=None, relax_hash=None):
    """SURVEY.md section 8e on one GPU: the C3 posterior stage and one
    consistency round with 8 virtual shards (mlp_set_shards; real N > 1 GPUs
    are unmeasured here), timing the all-gathers of the sparse set (every
    shard pulls every other shard's block on its own copy streams, the parent
    takes the full store) -- device-to-device copies here, peer copies over
    xGMI on a multi-GPU box."""
    from mlprobs_amd.engine import Family
    fam = Family(seqs, shards=8)
    # the library's default budget: the 8 shards split it less room for their
    # 9 store copies and gather buffers (round 4 set 120 GiB here: with the
    # whole default split, the device ran full and the gather took 411 ms
    # against 17 ms)
    # twice: the first stage allocates the shards' scratch and store copies
    # (a fresh allocation can stall ~5.7 s while the driver releases what the
    # bench's own stage freed), the second is warm
    runs = []
    for _ in range(2):
        fam.profile(True)
        t0 = time.perf_counter()
        fam.posteriors(args.pid, args.delta)
        fam.synchronize()
        runs.append((time.perf_counter() - t0, fam.kernel_times()['allgather']['ms']))
    t_post, gms = runs[1]
    kt = {'ms': gms}
    sh_post = store_hash(fam)
    rp, eo, cols, vals = fam.export()
    store_bytes = int(eo[-1]) * 6 + rp.nbytes
    res = {'shards': 8, 'posterior_stage_s': t_post, 'gather_ms': kt['ms'], 'store_bytes': store_bytes,
           'bytes_moved': 9 * store_bytes, 'cold_posterior_stage_s': runs[0][0], 'cold_gather_ms': runs[0][1],
           'note': '8 destinations x the whole store + the parent\'s copy; virtual shards share one GPU; '
                   'the second (warm) of two posterior stages, the first as cold_*'}
    fam.profile(True)
    t0 = time.perf_counter()
    fam.relax(1)
    fam.synchronize()
    res['relax_round_s'] = time.perf_counter() - t0
    res['relax_gather_ms'] = fam.kernel_times()['allgather']['ms']  # counters reset before the round
    sh_relax = store_hash(fam)
    # the sharded run must equal the unsharded one bit for bit (store,
    # distances, MEA scores, entry counts; posterior stage and round 1)
    res['identical_to_unsharded'] = {'posterior_stage': None if post_hash is None else sh_post == post_hash,
                                     'relax_round1': None if relax_hash is None else sh_relax == relax_hash}
    fam.close()
    for k, v in res['identical_to_unsharded'].items():
        if v is False:
            raise SystemExit(f'8 virtual shards: {k} differs from the unsharded run')
    log(f"shards: posteriors {t_post:.2f} s (gather {kt['ms']:.1f} ms), relax round {res['relax_round_s']:.2f} s")
    return res


def hbm_stream():
    """The on-box HBM bandwidth (tools/probe/hbm_stream: 16-byte read, write
    and copy kernels over 8 GiB, best of 10): the measured peak each roofline
    is also quoted against."""
    probe = os.path.join(ROOT, 'tools', 'probe', 'hbm_stream')
    if not os.path.exists(probe):
        return None
    r = subprocess.run([probe, '8', '10'], capture_output=True, text=True, timeout=120)
    if r.returncode != 0:
        return {'error': r.stderr[-300:]}
    s = json.loads(r.stdout.strip().splitlines()[-1])
    s['peak_GBps'] = max(s['read_gbps'], s['write_gbps'], s['copy_gbps'])
    log(f"hbm stream: read {s['read_gbps']:.0f} write {s['write_gbps']:.0f} copy {s['copy_gbps']:.0f} GB/s")
    return s


def c5_pipeline(args):
    """C5 (BASELINE.json configs[4]): the whole MLProbs pipeline per family
    -- features, classifier 1, c_p_np_aln -p 0|1, column scores, classifiers
    3/2, region split, quickprobs on every region kept if not worse, combine,
    fallbacks -- as `mlprobs_amd/cli/mlprobs`, one process per family (as
    MLProbs.py runs), aligners in-process (host context up to 4e6 pair-cells,
    one device context above: the default dispatch), over EVERY TEST/ox +
    TEST/sabre family (818, inputs from tests/golden/sweep.json.xz), one after
    another, as the reference's harness times them (script.py:42-60: every
    family of a benchmark, mean seconds).  Baseline: the same orchestration
    driving the reference CLIs built from source as external commands,
    exactly as MLProbs.py spawns them (c_p_np_aln with its own thread count
    and passive OpenMP waits, quickprobs -t --cpu-threads) on the same
    families; the reference's Python orchestration itself (not on the box) is
    not in that time, so the baseline is a lower bound of the reference
    pipeline's.  Times are split by the path the family took (trace
    `device_runs`).  Readouts: MLProbs' SP score (un_sp) of each final MSA and
    TC against the published MLProbs output of the family (output4evaluation/,
    tests/golden/c5_published.json.xz), and how many outputs equal the
    reference CLIs' (the reference's multi-threaded quickprobs makes this
    informative only; byte parity at every stage is pinned by
    tests/test_pipeline.py and tests/test_heavy_gpu.py).  The -p 1
    refinement reseeds rand() with srand(time(0)) (CPNP/MSA.cpp:1896), so
    every run here -- ours, the reference CLIs', the batch leg's -- reads
    one fixed clock (C5_CLOCK: MLP_SRAND_TIME for ours, the reference built
    with oracle/fixtime.c as _ref/c_p_np_aln_ft); at the wall clock two runs
    of the same family a second apart differ on -p 1 families."""
    import hashlib
    import lzma
    bin_ = os.path.join(ROOT, 'mlprobs_amd', 'cli', 'mlprobs')
    ref_cp = os.path.join(ROOT, 'oracle', '_ref', 'c_p_np_aln_ft')
    if not os.path.exists(ref_cp):
        ref_cp = os.path.join(ROOT, 'oracle', '_ref', 'c_p_np_aln')
    ref_qp = os.path.join(ROOT, 'oracle', '_ref', 'quickprobs')
    if not os.path.exists(bin_):
        return None
    with lzma.open(os.path.join(ROOT, 'tests', 'golden', 'sweep.json.xz'), 'rt') as fh:
        fams = json.load(fh)
    pub_path = os.path.join(ROOT, 'tests', 'golden', 'c5_published.json.xz')
    pub = {}
    if os.path.exists(pub_path):
        with lzma.open(pub_path, 'rt') as fh:
            pub = json.load(fh)
    names = [k for k in sorted(fams) if k.split('/')[0] in ('ox', 'sabre')]
    if args.c5_stride > 1:
        names = names[::args.c5_stride]
    with_ref = os.path.exists(ref_cp) and os.path.exists(ref_qp) and not args.no_cpu and args.c5_ref != 'none'
    ref_names = set(names)
    if args.c5_ref == 'sample':
        # every 8th family below 5e7 pair-cells: the reference CLIs take 100-110 s on each of the five
        # families above it (profiles/r04i_c5_full.json holds the run over every family)
        ref_names = {k for k in names[::8] if fams[k]['cells'] < 5e7}
    attribution = {}
    att_path = os.path.join(ROOT, 'profiles', C5_ATTRIBUTION)
    if os.path.exists(att_path):
        with open(att_path) as fh:
            attribution = {r['family']: r['cause'] for r in json.load(fh)['rows'] if r.get('cause')}
    last_log = time.perf_counter()
    recs, calls, paths, fails, same, differ = [], 0, {}, 0, 0, []
    sp_o, sp_r, sp_p, tc_o, tc_r = [], [], [], [], []
    env_ref = dict(os.environ, OMP_NUM_THREADS=str(args.cpu_threads), OMP_WAIT_POLICY='passive',
                   REF_FIXED_TIME=C5_CLOCK)
    env_ours = dict(os.environ, MLP_SRAND_TIME=C5_CLOCK)
    t_start = time.perf_counter()
    with tempfile.TemporaryDirectory() as td:
        for k, name in enumerate(names):
            if k % 50 == 0 or time.perf_counter() - last_log > 20:
                log(f'c5 family {k}/{len(names)} {name} ({time.perf_counter() - t_start:.0f} s)')
                last_log = time.perf_counter()
            e = fams[name]
            fa = os.path.join(td, 'f.fa')
            with open(fa, 'wb') as fh:
                fh.write(e['fa'].encode('latin-1'))
            out, trace = os.path.join(td, 'o.msa'), os.path.join(td, 't.json')
            t0 = time.perf_counter()
            r = subprocess.run([bin_, '-q', '--trace', trace, fa, out], capture_output=True, timeout=900, env=env_ours)
            rec = {'name': name, 'cells': e['cells'], 's': time.perf_counter() - t0, 'device': False, 'ref_s': None}
            recs.append(rec)
            if r.returncode != 0:
                fails += 1
                continue
            with open(out, encoding='latin-1') as fh:
                mine = fh.read()
            with open(trace) as fh:
                tr = json.load(fh)
            rec['device'] = tr.get('device_runs', 0) > 0
            rec['sha1'] = hashlib.sha1(mine.encode('latin-1')).hexdigest()
            calls += tr['quickprobs_calls']
            paths[tr['path']] = paths.get(tr['path'], 0) + 1
            sp_o.append(sp_score(mine))
            if name in pub:
                sp_p.append(sp_score(pub[name]))
                tc_o.append(tc_score(mine, pub[name]))
            if with_ref and name in ref_names:
                log(f'c5 {name}: ours {rec["s"]:.2f} s, reference CLIs ...') if e['cells'] > 2e7 else None
                out2, trace2 = os.path.join(td, 'r.msa'), os.path.join(td, 'rt.json')
                t0 = time.perf_counter()
                subprocess.run([bin_, '-q', '--trace', trace2, '--cpnp', ref_cp, '--quickprobs',
                                f'{ref_qp} -t {args.cpu_threads}', '--tmp', td, fa, out2],
                               capture_output=True, timeout=1800, env=env_ref)
                rec['ref_s'] = time.perf_counter() - t0
                with open(out2, encoding='latin-1') as fh:
                    refo = fh.read()
                same += refo == mine
                if refo != mine:
                    # where the two runs part (mlprobs --trace stages); the
                    # reference CLIs run twice more on the family: outputs
                    # that disagree with each other (or one equal to ours)
                    # show the reference's own multi-threaded races (DESIGN.md
                    # section 2); else the cause committed for the family by
                    # tools/c5_attribution.py, if any
                    with open(trace2) as fh:
                        tr2 = json.load(fh)
                    stage = next((s for s in C5_STAGES[:-1] if tr.get(s) != tr2.get(s)), 'output')
                    reruns = []
                    for _ in range(2):
                        subprocess.run([bin_, '-q', '--cpnp', ref_cp, '--quickprobs', f'{ref_qp} -t {args.cpu_threads}',
                                        '--tmp', td, fa, out2], capture_output=True, timeout=1800, env=env_ref)
                        with open(out2, encoding='latin-1') as fh:
                            reruns.append(fh.read())
                    if any(x != refo for x in reruns):
                        cause = 'race: reference reruns ' + ('equal ours' if mine in reruns else 'disagree')
                    else:
                        cause = attribution.get(name, 'unexplained: reference reproducible')
                    differ.append({'name': name, 'path': tr['path'], 'first_stage': stage, 'cause': cause})
                sp_r.append(sp_score(refo))
                if name in pub:
                    tc_r.append(tc_score(refo, pub[name]))

    def mean(v):
        v = [x for x in v if x is not None]
        return float(np.mean(v)) if v else None

    def summary(sel):
        ours = [x['s'] for x in sel]
        out = {'families': len(sel), 'pair_cells': int(sum(x['cells'] for x in sel))}
        if ours:
            out.update(s_per_family={'median': float(np.median(ours)), 'mean': float(np.mean(ours)),
                                     'max': float(np.max(ours)), 'total': float(np.sum(ours))})
        both = [x for x in sel if x['ref_s'] is not None]
        if both:
            refs = [x['ref_s'] for x in both]
            mine = [x['s'] for x in both]
            out['reference_clis_s_per_family'] = {'families': len(both), 'median': float(np.median(refs)),
                                                  'mean': float(np.mean(refs)), 'total': float(np.sum(refs)),
                                                  'ours_on_these': {'median': float(np.median(mine)),
                                                                    'mean': float(np.mean(mine)),
                                                                    'total': float(np.sum(mine))}}
            out['speedup_mean'] = float(np.mean(refs)) / float(np.mean(mine))
            out['speedup_median'] = float(np.median(refs)) / float(np.median(mine))
        return out

    dev = [x for x in recs if x['device']]
    res = {'families': len(names), 'failed': fails,
           'sample': 'every TEST/ox + TEST/sabre family' if args.c5_stride <= 1 else
                     f'every {args.c5_stride}th TEST/ox + TEST/sabre family',
           'pipeline': 'mlprobs (MLProbs.py + utils/*.py restated in C++, aligners in-process, default dispatch)',
           'host_path_families': len(recs) - len(dev), 'device_path_families': len(dev),
           'quickprobs_region_calls': calls, 'paths': paths,
           'all': summary(recs), 'device_path': summary(dev), 'host_path': summary([x for x in recs if not x['device']]),
           'slowest': sorted(({'name': x['name'], 's': x['s'], 'ref_s': x['ref_s'], 'cells': x['cells']}
                              for x in recs), key=lambda x: -x['s'])[:8],
           'sp_un_sp_mean': mean(sp_o), 'published_sp_un_sp_mean': mean(sp_p),
           'tc_vs_published_mean': mean(tc_o), 'wall_s': time.perf_counter() - t_start}
    res['s_per_family'] = res['all'].get('s_per_family')
    res['clock'] = C5_CLOCK
    if with_ref:
        res['reference_clis'] = (f'the same orchestration driving oracle/_ref/{os.path.basename(ref_cp)} (its own thread count, '
                                 f'passive OpenMP waits) and oracle/_ref/quickprobs -t {args.cpu_threads} as external '
                                 f'commands, on {"every family" if args.c5_ref == "all" else "every 8th family below 5e7 pair-cells"} '
                                 '(speed-ups over the families both ran)')
        res['speedup_mean'] = res['all'].get('speedup_mean')
        res['speedup_median'] = res['all'].get('speedup_median')
        res['identical_to_reference_clis'] = same
        res['differing'] = differ
        res['reference_clis_families'] = len(sp_r)
        res['reference_clis_sp_un_sp_mean'] = mean(sp_r)
        res['reference_clis_tc_vs_published_mean'] = mean(tc_r)
    res['runs'] = recs
    log(f"c5: {len(recs)} families in {res['wall_s']:.0f} s, {len(dev)} on the device")
    return res


def c5_batch(args, devices, per_process=None):
    """C5 at family level over the GPUs (`mlprobs --batch`): one worker
    process per device, forked before any GPU call, each keeping one device
    context for all its families and taking the next family, largest first,
    from a shared counter; every TEST/ox + TEST/sabre family, outputs written
    as separate runs write them.  Wall time of the whole benchmark and the
    per-family seconds inside the workers; with the per-process leg's records
    (per_process), how many outputs are byte-identical to those runs'."""
    import hashlib
    import lzma
    bin_ = os.path.join(ROOT, 'mlprobs_amd', 'cli', 'mlprobs')
    if not os.path.exists(bin_):
        return None
    with lzma.open(os.path.join(ROOT, 'tests', 'golden', 'sweep.json.xz'), 'rt') as fh:
        fams = json.load(fh)
    names = [k for k in sorted(fams) if k.split('/')[0] in ('ox', 'sabre')]
    if args.c5_stride > 1:
        names = names[::args.c5_stride]
    with tempfile.TemporaryDirectory() as td:
        lines = []
        for k, name in enumerate(names):
            fa = os.path.join(td, f'f{k}.fa')
            with open(fa, 'wb') as fh:
                fh.write(fams[name]['fa'].encode('latin-1'))
            lines.append(f"{fa}\t{os.path.join(td, f'f{k}.msa')}\n")
        lst, rep = os.path.join(td, 'list.txt'), os.path.join(td, 'report.json')
        with open(lst, 'w') as fh:
            fh.writelines(lines)
        log(f'c5 batch: {len(names)} families over devices {devices}')
        t0 = time.perf_counter()
        r = subprocess.run([bin_, '-q', '--batch', lst, '--devices', devices, '--report', rep], capture_output=True,
                           timeout=1800, env=dict(os.environ, MLP_SRAND_TIME=C5_CLOCK))
        wall = time.perf_counter() - t0
        if not os.path.exists(rep):
            return {'error': r.stderr.decode(errors='replace')[-400:]}
        with open(rep) as fh:
            report = json.load(fh)
        sha = {}
        for k, name in enumerate(names):
            p = os.path.join(td, f'f{k}.msa')
            if os.path.exists(p):
                with open(p, 'rb') as fh:
                    sha[name] = hashlib.sha1(fh.read()).hexdigest()
    runs = report['runs']
    secs = [x['s'] for x in runs if x['status'] == 0]
    dev = [x['s'] for x in runs if x['status'] == 0 and x['device_runs'] > 0]
    res = {'families': len(names), 'devices': devices, 'workers': report['workers'], 'failed': report['failed'],
           'wall_s': wall, 'wall_s_inside': report['wall_s'],
           's_per_family': {'median': float(np.median(secs)), 'mean': float(np.mean(secs)),
                            'total': float(np.sum(secs))} if secs else None,
           'device_path': {'families': len(dev), 'median': float(np.median(dev)), 'mean': float(np.mean(dev))}
           if dev else None,
           'mode': 'mlprobs --batch: one worker process per device, one context per worker, largest family first'}
    if per_process:
        pp = {x['name']: x.get('sha1') for x in per_process}
        both = [n for n in names if n in sha and pp.get(n)]
        res['identical_to_per_process'] = sum(sha[n] == pp[n] for n in both)
        res['compared'] = len(both)
        res['differing_from_per_process'] = [n for n in both if sha[n] != pp[n]][:20]
    log(f"c5 batch: {len(names)} families in {wall:.1f} s ({report['workers']} workers), "
        f"{res.get('identical_to_per_process')} of {res.get('compared')} identical to the per-process runs")
    return res


def quickprobs_stage(fam, fam_in, total_cells, args):
    """QuickProbs' posterior stage (MLP_PID_QP) and one consistency round
    (its default for N > 50) on the same family, resident in HBM; the
    reference QuickProbs posterior stage (oracle/_ref/qp_probe, compiled from
    the reference sources) timed on a bounded sample as its CPU baseline."""
    from mlprobs_amd.engine import PID_QP
    fam.profile(False)
    fam.posteriors(PID_QP, 0.0)  # warm-up
    fam.synchronize()
    t0 = time.perf_counter()
    fam.posteriors(PID_QP, 0.0)
    fam.synchronize()
    dt = time.perf_counter() - t0
    tr = time.perf_counter()
    fam.relax_qp(1, np.ones(fam.n, np.float32))
    fam.synchronize()
    dr = time.perf_counter() - tr
    res = {'posterior_pair_cells_per_s': total_cells / dt, 'posterior_ms': dt * 1e3,
           'consistency_round_s': dr, 'nnz_out': int(fam.results()[2].sum())}
    probe = os.path.join(ROOT, 'oracle', '_ref', 'qp_probe')
    if os.path.exists(probe) and not args.no_cpu:
        with tempfile.TemporaryDirectory() as td:
            path = os.path.join(td, 'fam.txt')
            with open(path, 'w') as fh:
                fh.write('\n'.join(sq for _, sq in fam_in))
            out = subprocess.run([probe, 'bench', path, str(args.cpu_pairs // 2), str(args.cpu_threads)],
                                 capture_output=True, text=True, timeout=600)
        if out.returncode == 0:
            r = json.loads(out.stdout.strip().splitlines()[-1])
            res['cpu_baseline'] = {'value': r['pair_cells_per_s'], 'unit': 'pair-cells/s',
                                   'cores': args.cpu_threads, 'kind': 'reference',
                                   'sample': f"first {r['pairs']} pairs, {r['seconds']:.1f} s, reference "
                                             "QuickProbs PosteriorStage::computePairwise"}
            res['speedup_vs_cpu'] = res['posterior_pair_cells_per_s'] / r['pair_cells_per_s']
    return res


def _r(x, sig=4):
    """Floats to `sig` significant digits, recursively (the printed line)."""
    if isinstance(x, float):
        return float(f'{x:.{sig}g}')
    if isinstance(x, dict):
        return {k: _r(v, sig) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_r(v, sig) for v in x]
    return x


def _pick(d, *keys):
    return {k: d[k] for k in keys if d is not None and k in d}


def compact_e2e(e2e):
    """Per end-to-end leg: median / max / every run's wall seconds, the median
    run's stage split, the drop-in's posterior stage and the output check."""
    out = {}
    for tag, rec in e2e.items():
        c = _pick(rec, 'median_s', 'max_s', 'runs_s', 'exit')
        c['stages_s'] = {k: v for k, v in rec.get('stages_s', {}).items() if v >= 0.005}
        if rec.get('outliers'):
            c['outliers'] = [_pick(o, 'run', 's', 'stage') for o in rec['outliers']]
        if 'posterior_stage' in rec:
            c['posterior_stage'] = _pick(rec['posterior_stage'], 'median_s', 'pair_cells_per_s')
        if 'reference_output' in rec:
            c['reference_output'] = _pick(rec['reference_output'], 'identical', 'tc_vs_reference')
        if 'reference_cpu' in rec:
            c['reference_cpu'] = _pick(rec['reference_cpu'], 'seconds', 'threads', 'identical_output')
        out[tag] = c
    return out


def compact_c5(c5):
    c = _pick(c5, 'families', 'failed', 'device_path_families', 'host_path_families', 'quickprobs_region_calls',
              'paths', 'speedup_mean', 'speedup_median', 'identical_to_reference_clis', 'reference_clis_families',
              'sp_un_sp_mean', 'published_sp_un_sp_mean', 'tc_vs_published_mean',
              'reference_clis_tc_vs_published_mean', 'wall_s', 'devices', 'scaling', 'clock')
    for k in ('all', 'device_path', 'host_path'):
        if k in c5:
            s = dict(c5[k].get('s_per_family', {}))
            r = c5[k].get('reference_clis_s_per_family')
            if r:
                s['reference_clis_mean'] = r['mean']
                s['ours_mean_on_reference_families'] = r['ours_on_these']['mean']
            c[k] = s
    if 'differing' in c5:
        d = c5['differing']
        causes = {}
        for x in d:
            causes[x['cause']] = causes.get(x['cause'], 0) + 1
        c['differing'] = {'n': len(d), 'causes': causes,
                          'first_stage': {s: sum(x['first_stage'] == s for x in d) for s in C5_STAGES
                                          if any(x['first_stage'] == s for x in d)},
                          'unexplained': [x['name'] for x in d if x['cause'].startswith('unexplained')][:12]}
    return c


def compact_relax(rx):
    c = _pick(rx, 'rounds', 'seconds', 'nnz_per_round', 'speedup_vs_cpu')
    c['per_round'] = [{'s': r['seconds'], 'relax_ms': r.get('kernels_ms', {}).get('relax'),
                       'nnz_out': r['nnz_out']} if 'ranks' not in r else
                      {'s': r['seconds'], 'gather_ms': r['gather_ms'], 'nnz_out': r['nnz_out'],
                       'ranks': [{'rank': q['rank'], 's': q['seconds'], 'relax_ms': q['relax_kernel_ms'],
                                  'gather_ms': q['gather_ms'], 'store_hash': q['store_hash'][:16]}
                                 for q in r['ranks']]}
                      for r in rx.get('per_round', [])]
    if 'round1' in rx:
        c['round1'] = _pick(rx['round1'], 'kernel_ms', 'macs_reference', 'mac_per_s')
    if 'roofline' in rx:
        c['roofline'] = _pick(rx['roofline'], 'bound', 'kernel', 'achieved', 'peak', 'unit', 'frac', 'traffic',
                              'avg_launch_ms', 'frac_of_measured')
    if 'cpu_baseline' in rx:
        c['cpu_baseline'] = rx['cpu_baseline']
    if 'parity' in rx:
        c['parity'] = _pick(rx['parity'], 'pairs', 'max_rel_err', 'violations', 'bit_exact')
    return c


def compact_line(out):
    """The one JSON line the driver parses: the headline keys, config,
    roofline, cpu_baseline, parity and summaries of every leg; the per-run
    and per-family detail stays in the side file (DETAIL_PATH).  Sections
    are dropped, least important first, if the line would pass LINE_LIMIT."""
    line = {k: v for k, v in out.items() if k not in ('e2e', 'c5_pipeline', 'c5_batch', 'relax', 'ranks',
                                                       'hbm_stream', 'virtual_shards', 'parity')}
    if out.get('parity'):
        line['parity'] = _pick(out['parity'], 'pairs', 'max_rel_err', 'violations', 'inexact',
                               'symmetric_difference', 'distance_max_rel_err', 'bit_exact')
    if out.get('hbm_stream') and 'peak_GBps' in out['hbm_stream']:
        line['hbm_stream'] = _pick(out['hbm_stream'], 'read_gbps', 'write_gbps', 'copy_gbps')
    if out.get('relax'):
        line['relax'] = compact_relax(out['relax'])
    if out.get('virtual_shards'):
        line['virtual_shards'] = {k: v for k, v in out['virtual_shards'].items() if k not in ('note', 'store_bytes', 'pool')}
    if out.get('ranks'):
        line['ranks'] = [{'rank': r['rank'], 'pairs': r['pairs'], 'step_ms': r['step_ms'],
                          'gather_ms': r['gather_ms'], 'gather_GBps': r['gather_GBps'],
                          'gather_bytes_in': r['gather_bytes_in'],
                          'roofline_frac': (r.get('roofline') or {}).get('frac'),
                          'store_hash': r['store_hash'][:16]} for r in out['ranks']]
    if out.get('c5_pipeline'):
        line['c5_pipeline'] = compact_c5(out['c5_pipeline'])
    if out.get('c5_batch'):
        line['c5_batch'] = {k: v for k, v in out['c5_batch'].items() if k != 'mode'}
    if out.get('e2e'):
        line['e2e'] = compact_e2e(out['e2e'])
    line['detail'] = os.path.relpath(DETAIL_PATH, ROOT) if DETAIL_PATH.startswith(ROOT) else DETAIL_PATH
    line = dict(_r(line), value=out['value'], ms_per_step=out['ms_per_step'])
    for drop in ('hbm_stream', 'e2e', 'c5_pipeline', 'virtual_shards', 'quickprobs', 'ranks'):
        if len(json.dumps(line)) <= LINE_LIMIT:
            break
        log(f'bench line over {LINE_LIMIT} bytes: {drop} left to {line["detail"]}')
        line.pop(drop, None)
    return line


def emit(out):
    """Full record to the side file, its summaries to stderr, the compact line
    to stdout."""
    os.makedirs(os.path.dirname(DETAIL_PATH), exist_ok=True)
    with open(DETAIL_PATH, 'w') as fh:
        json.dump(out, fh)
    for tag, rec in (out.get('e2e') or {}).items():
        log(f'e2e {tag}: runs ' + ', '.join(f"{x['s']:.2f}" for x in rec.get('runs', [])) + ' s; median stages ' +
            ', '.join(f'{k} {v:.3f}' for k, v in rec.get('stages_s', {}).items() if v >= 0.01))
    c5 = out.get('c5_pipeline')
    if c5:
        for x in c5.get('slowest', []):
            log(f"c5 slow: {x['name']} {x['s']:.2f} s ({x['cells']:.3g} pair-cells)")
        for x in c5.get('differing', []):
            log(f"c5 differs from the reference CLIs: {x['name']} ({x['path']}): first at {x['first_stage']}, "
                f"cause {x['cause']}")
    line = compact_line(out)
    s = json.dumps(line)
    log(f'bench line {len(s)} bytes; full record {DETAIL_PATH}')
    print(s, flush=True)


def main():
    args = parse()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        if args.host:
            dist.init_process_group('gloo')
        else:
            torch.cuda.set_device(local)
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    from mlprobs_amd import synth
    from mlprobs_amd.engine import Family

    # end-to-end family timings first, on an idle device (a process that
    # follows a large release waits for the driver to clear that memory)
    log('start')
    if args.only_c5:
        c5 = c5_pipeline(args)
        print(json.dumps({'c5_pipeline': _r(compact_c5(c5))}))
        os.makedirs(os.path.dirname(DETAIL_PATH), exist_ok=True)
        with open(DETAIL_PATH, 'w') as fh:
            json.dump({'c5_pipeline': c5}, fh)
        return
    stream = hbm_stream() if (world == 1 and not args.host) else None
    e2e = e2e_families(args) if (not args.no_e2e and world == 1) else None
    c5 = c5_pipeline(args) if (not args.no_e2e and not args.no_c5 and world == 1 and rank == 0) else None
    c5b = c5_batch(args, '0', c5.get('runs') if c5 else None) \
        if (not args.no_e2e and not args.no_c5 and world == 1 and rank == 0 and not args.host) else None
    if args.relax < 0:
        args.relax = 4 if world == 1 else 1
    fam_in = synth.family(args.n, args.len, args.s, seed=args.seed)
    seqs = [s for _, s in fam_in]
    lens = np.array([len(s) for s in seqs], np.int64)
    fam = Family(seqs, host=True) if args.host else Family(seqs, device=local if world > 1 else 0)
    if world > 1 and not args.host:
        uid = Family.unique_id() if rank == 0 else None
        obj = [uid]
        dist.broadcast_object_list(obj, src=0)
        fam.comm_init(obj[0], world, rank)
    p0, p1 = fam.shard(world, rank)
    ex = RankExchange(fam, world, rank, dist, args.host) if world > 1 else None
    total_cells = 0
    for a in range(args.n):
        total_cells += int(((lens[a] + 1) * (lens[a + 1:] + 1)).sum())

    def step():
        fam.posteriors(args.pid, args.delta, p0, p1)
        if world > 1:
            ex.gather(p0, p1)

    def barrier():
        fam.synchronize()
        if world > 1:
            if not args.host:
                import torch
                torch.cuda.synchronize()
            dist.barrier()

    log('posterior stage')
    for _ in range(args.warmup):
        fam.profile(False)
        step()
    fam.profile(True)
    if ex:
        ex.reset()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    dt = time.perf_counter() - t0
    dt_rank = dt
    if world > 1:
        import torch
        t = torch.tensor([dt], dtype=torch.float64, device='cpu' if args.host else 'cuda')
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    kt = fam.kernel_times()
    ranks_info, relax_multi = None, None
    if world > 1:
        log('per-rank records and consistency rounds')
        ranks_info, relax_multi = multirank_legs(fam, ex, args, world, rank, dist, lens, p0, p1, dt_rank, kt, barrier)
    gpu_dist, _, nnz = fam.results()  # posterior-stage sparse set (before any relaxation)
    gpu_dist, nnz = gpu_dist.copy(), nnz.copy()
    # the posterior store, kept for the same-run parity readouts (rank 0)
    post_store = [a.copy() for a in fam.export()] if (rank == 0 and world == 1 and not args.no_cpu) else None
    post_hash = store_hash(fam) if (world == 1 and not args.no_shards) else None
    log('relaxation rounds')
    relax_info = relax_leg(fam, args, args.n, lens, total_cells) if (args.relax > 0 and world == 1) else None
    value = total_cells * args.steps / dt
    # roofline of the dominant kernel (largest accumulated device time)
    dom = max(ALGO_BYTES, key=lambda k: kt[k]['ms'])
    launches = max(kt[dom]['launches'], 1)
    avg_ms = kt[dom]['ms'] / launches
    bytes_per_launch = ALGO_BYTES[dom] * kt[dom]['cells'] / launches
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    # measured HBM bytes and VALU instructions per pair-cell of this kernel
    # group from the committed PMC passes (tools/pmc_run.sh), scaled to the
    # cells of one launch here
    traffic, valu = None, None
    pmc = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')
    if os.path.exists(pmc) and avg_ms > 0:
        with open(pmc) as fh:
            g = json.load(fh).get(dom)
        if g:
            cells_per_launch = kt[dom]['cells'] / launches
            traffic = g['traffic_bytes_per_cell'] * cells_per_launch / 1e9
            issued = g['valu_insts_per_cell'] * cells_per_launch / (avg_ms * 1e-3)
            # against the group's mix-weighted issue peak (its full / half-rate
            # instruction mix, tools/valu_mix.py) and the
            # all-full-rate 1.23e12 beside it
            mix = g.get('valu_mix_peak') or VALU_PEAK_WAVE_INSTS
            valu = {'achieved': issued, 'peak': mix, 'unit': 'wave-instr/s', 'frac': issued / mix,
                    'peak_all_full_rate': VALU_PEAK_WAVE_INSTS, 'frac_of_full_rate': issued / VALU_PEAK_WAVE_INSTS,
                    'insts_per_cell': g['valu_insts_per_cell'], 'source': 'profiles/pmc_traffic.json'}
    log('quickprobs stage')
    qp_info = quickprobs_stage(fam, fam_in, total_cells, args) if (world == 1 and not args.no_qp and not args.host) else None
    shards_info = None
    if world == 1 and not args.no_shards and not args.host:
        # the main context's batch scratch (most of the device) goes first: the
        # 8 shard contexts need their own.  The bench is a long-lived caller
        # creating one context after another, so the process pool keeps the
        # closing family's blocks for the shards (MLP_POOL_KEEP_GB; the
        # default 32 GiB cap would hand them to the driver and the shards'
        # first allocations would wait for it to clear them, DESIGN.md
        # section 3), and gives them back after the leg
        from mlprobs_amd import engine
        os.environ['MLP_POOL_KEEP_GB'] = '1000000'
        fam.close()
        fam = None
        log('virtual shards')
        try:
            shards_info = shard_gather(args, seqs, post_hash, relax_info['round1_hash'] if relax_info else None)
        finally:
            os.environ.pop('MLP_POOL_KEEP_GB', None)
            engine.pool_trim(0)
        shards_info['pool'] = 'the main family\'s blocks kept for the shard contexts'
    if world > 1 and not args.host and not args.no_c5 and not args.no_e2e:
        # C5 at family level over all N GPUs: the ranks release their
        # contexts first, then rank 0's workers take one device each
        fam.close()
        fam = None
        barrier_host = dist.barrier
        barrier_host()
        if rank == 0:
            c5b = c5_batch(args, ','.join(str(d) for d in range(world)))
        barrier_host()
    out = None
    if rank == 0:
        cpu, parity = None, None
        if not args.no_cpu and world == 1:
            with tempfile.TemporaryDirectory() as td:
                fa = os.path.join(td, 'fam.fa')
                synth.write_fasta(fa, fam_in)
                log('cpu baseline')
                cpu, parity = cpu_baseline(fa, args, args.n, lens, post_store, gpu_dist)
            post_store = None
        out = {
            'metric': METRIC,
            'value': value,
            'unit': 'pair-cells/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': dt / args.steps * 1e3,
            'higher_is_better': True,
            'scaling': 'strong',
            'vs_baseline': None,
            'dtype': 'f32',
            'data': 'synthetic',
            'config': {'workload': f'C3 all-pairs posterior stage: {args.n} seqs x {args.len} aa synthetic '
                                   f'(s={args.s}, seed {args.seed}), pid {args.pid} '
                                   '(5-state HMM + partition function + local HMM, RMS merge, MEA, sparsify)',
                       'n_seqs': args.n, 'length': args.len, 'pairs': int(args.n * (args.n - 1) // 2),
                       'pair_cells': int(total_cells), 'nnz': int(nnz.sum()),
                       'parallelism': f'pair-sharded dp{world}' + (' + RCCL all-gather' if world > 1 else '')},
            'roofline': {'bound': 'hbm', 'kernel': dom, 'achieved': achieved, 'peak': HBM_PEAK_GBS,
                         'unit': 'GB/s', 'frac': achieved / HBM_PEAK_GBS, 'traffic': traffic,
                         'traffic_unit': 'GB per launch (2 x FETCH_SIZE + WRITE_SIZE)',
                         'algo_bytes_per_cell': ALGO_BYTES[dom], 'avg_launch_ms': avg_ms,
                         'valu_issue': valu},
            'stage_roofline': {'algo_bytes_per_cell': STAGE_BYTES,
                               'achieved_GBps': value * STAGE_BYTES / 1e9,
                               'frac': value * STAGE_BYTES / 1e9 / HBM_PEAK_GBS},
            'kernels_ms_per_step': {k: v['ms'] / args.steps for k, v in kt.items() if v['launches']},
            'batches_per_step': kt['forward']['launches'] / args.steps,
            'cpu_baseline': cpu,
            'parity': parity,
        }
        if cpu:
            out['speedup_vs_cpu'] = value / cpu['value']
        if stream and 'peak_GBps' in stream:
            mp = stream['peak_GBps']
            out['hbm_stream'] = stream
            out['roofline']['peak_measured'] = mp
            out['roofline']['frac_of_measured'] = achieved / mp
            out['stage_roofline']['frac_of_measured'] = value * STAGE_BYTES / 1e9 / mp
            if relax_info:
                relax_info['roofline']['peak_measured'] = mp
                relax_info['roofline']['frac_of_measured'] = relax_info['roofline']['achieved'] / mp
        if relax_info:
            out['relax'] = relax_info
        if e2e is not None:
            out['e2e'] = e2e
        if c5 is not None:
            out['c5_pipeline'] = c5
        if c5b is not None:
            out['c5_batch'] = c5b
        if qp_info is not None:
            out['quickprobs'] = qp_info
        if shards_info is not None:
            out['virtual_shards'] = shards_info
        if ranks_info is not None:
            out['ranks'] = ranks_info
            out['gather_ms'] = max(r['gather_ms'] for r in ranks_info)
            moved = sum(r['gather_bytes_in'] for r in ranks_info)
            out['gather_GBps'] = moved / (out['gather_ms'] * 1e-3) / 1e9 if out['gather_ms'] > 0 else None
            out['gather_note'] = ('per step: max over ranks of the all-gather time; gather_GBps = bytes all ranks '
                                  'received / that time' + (' (host dry run over gloo)' if args.host else
                                                            ' (RCCL over xGMI)'))
            out['ranks_identical'] = len({r['store_hash'] for r in ranks_info}) == 1 and all(
                len({r['store_hash'] for r in rr['ranks']}) == 1 for rr in (relax_multi or {}).get('per_round', []))
            if relax_multi is not None:
                out['relax'] = relax_multi
            if args.host:
                out['data'] = 'synthetic (host contexts over gloo: CPU dry run, not a GPU measurement)'
        emit(out)
    if fam is not None:
        fam.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
