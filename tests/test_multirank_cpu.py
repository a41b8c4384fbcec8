"""Multi-rank path on CPU (gloo): the pair sharding and the all-gather layout
of libmlpgpu (mlp_shard_plan / mlp_gather_layout, the host logic behind
mlp_shard_range and mlp_allgather) with real process-group exchange.

Each rank computes the posteriors of its own shard with the library itself
(its host context, mlp_ctx_create_host: the product's pair body on host
threads, no GPU here), the ranks exchange (p0, p1, entries) and their CSR
blocks over gloo, place them where the library's layout says, and every rank
must end up with the single-process store of the oracle, the checker
(bit-identical results for any rank count).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'oracle'))

DELTA = 0.132548


def _family():
    from mlprobs_amd import synth
    fam = [s for _, s in synth.family(7, 40, 0.6, seed=23)]
    fam[2] = fam[2][:17]   # ragged lengths
    fam[5] = fam[5] + fam[1][:9]
    return fam


def _pair_block(m, s1, s2, pid):
    import orc
    post = orc.pair_posterior(m, s1, s2, pid)
    rp, cols, vals = orc.sparsify(len(s1), len(s2), post)
    score = orc.mea(len(s1), len(s2), post)
    dist_ = np.float32(1.0) - np.float32(score) / np.float32(min(len(s1), len(s2)))
    return rp.astype(np.int32), cols.astype(np.uint16), vals.astype(np.float32), np.float32(dist_)


def _store(fam, pid, p0, p1):
    """Canonical CSR pieces of pairs [p0, p1): row_ptr blocks, entries, distances."""
    import orc
    from mlprobs_amd.engine import pairs_of
    m = orc.model(DELTA)
    rps, cols, vals, dists = [], [], [], []
    for a, b in pairs_of(len(fam))[p0:p1]:
        rp, c, v, d = _pair_block(m, fam[a], fam[b], pid)
        rps.append(rp)
        cols.append(c)
        vals.append(v)
        dists.append(d)
    cat = lambda xs, dt: np.concatenate(xs) if xs else np.zeros(0, dt)
    return cat(rps, np.int32), cat(cols, np.uint16), cat(vals, np.float32), np.array(dists, np.float32)


def _store_lib(fam, pid, p0, p1):
    """The same pieces from libmlpgpu's host context over pairs [p0, p1)."""
    from mlprobs_amd.engine import Family
    f = Family(fam, host=True)
    try:
        f.posteriors(pid, DELTA, p0, p1)
        rp_full, eo, cols, vals = f.export()
        d, _, _ = f.results(p0, p1)
        rp = rp_full[f.rp_off[p0]:f.rp_off[p1]].astype(np.int32)
        e0, e1 = int(eo[p0]), int(eo[p1])
        return rp, cols[e0:e1].copy(), vals[e0:e1].copy(), d.astype(np.float32)
    finally:
        f.close()


def _worker(rank, world, port, pid, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from mlprobs_amd import engine
        fam = _family()
        lens = np.array([len(s) for s in fam], np.int32)
        P = len(fam) * (len(fam) - 1) // 2
        p0, p1 = engine.shard_plan(lens, world, rank)
        rp, cols, vals, dists = _store_lib(fam, pid, p0, p1)
        shards = [None] * world
        dist.all_gather_object(shards, (p0, p1, int(len(cols))))
        ebase = engine.gather_layout(P, shards)
        blocks = [None] * world
        dist.all_gather_object(blocks, (rp, cols, vals, dists))
        # place every rank's block where mlp_allgather puts it
        total = int(ebase[-1])
        g_cols = np.zeros(total, np.uint16)
        g_vals = np.zeros(total, np.float32)
        g_rp = np.concatenate([b[0] for b in blocks])
        g_d = np.concatenate([b[3] for b in blocks])
        for r, b in enumerate(blocks):
            g_cols[ebase[r]:ebase[r + 1]] = b[1]
            g_vals[ebase[r]:ebase[r + 1]] = b[2]
        q.put((rank, shards, g_rp, g_cols, g_vals, g_d))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.mark.parametrize('world,pid', [(2, 2), (3, 0)])
def test_sharded_store_matches_single_process(world, pid):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, pid, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    fam = _family()
    P = len(fam) * (len(fam) - 1) // 2
    rp, cols, vals, dists = _store(fam, pid, 0, P)
    for rank, shards, g_rp, g_cols, g_vals, g_d in got:
        # shards tile [0, P) and are balanced by cells
        assert shards[0][0] == 0 and shards[-1][1] == P
        assert all(shards[r][1] == shards[r + 1][0] for r in range(world - 1))
        assert np.array_equal(g_rp, rp)
        assert np.array_equal(g_cols, cols)
        assert np.array_equal(g_vals, vals)
        assert np.array_equal(g_d, dists)


def test_shard_plan_balance():
    from mlprobs_amd import engine
    rng = np.random.default_rng(5)
    lens = rng.integers(20, 600, size=61).astype(np.int32)
    n = len(lens)
    cost = np.array([(lens[a] + 1) * (lens[b] + 1) for a in range(n) for b in range(a + 1, n)], np.float64)
    for R in (1, 2, 4, 8):
        cuts = [engine.shard_plan(lens, R, r) for r in range(R)]
        assert cuts[0][0] == 0 and cuts[-1][1] == len(cost)
        for r in range(R - 1):
            assert cuts[r][1] == cuts[r + 1][0]
        loads = [cost[a:b].sum() for a, b in cuts]
        assert max(loads) - cost.sum() / R <= cost.max() + 1e-6


def test_gather_layout_rejects_gaps():
    from mlprobs_amd import engine
    assert list(engine.gather_layout(10, [(0, 3, 5), (3, 10, 2)])) == [0, 5, 7]
    with pytest.raises(engine.MlpError):
        engine.gather_layout(10, [(0, 3, 5), (4, 10, 2)])
    with pytest.raises(engine.MlpError):
        engine.gather_layout(10, [(0, 3, 5), (3, 9, 2)])


# ---- consistency rounds: output pairs split by estimated multiply-adds
ROUNDS = 2


def _relax_worker(rank, world, port, q):
    """One rank of the sharded consistency rounds, all in the library: the
    posterior stage on its host context, then per round its MAC-balanced
    output range (mlp_relax_shard_plan) relaxed by mlp_relax_range, the
    blocks exchanged over gloo and placed with the library's gather layout,
    and the gathered store imported back (mlp_csr_import) for the next
    round -- what mlp_allgather does over RCCL."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from mlprobs_amd import engine
        from mlprobs_amd.engine import Family
        fam = _family()
        lens = np.array([len(s) for s in fam], np.int32)
        P = len(fam) * (len(fam) - 1) // 2
        f = Family(fam, host=True)
        try:
            f.posteriors(0, DELTA)
            rounds = []
            for _ in range(ROUNDS):
                _, eo, _, _ = f.export()
                bounds = engine.relax_shard_plan(lens, np.diff(eo), world)
                r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
                f.relax_range(r0, r1)
                rp_full, eo, cols, vals = f.export()
                rp = rp_full[f.rp_off[r0]:f.rp_off[r1]].astype(np.int32)
                blk = (rp, cols[int(eo[r0]):int(eo[r1])].copy(), vals[int(eo[r0]):int(eo[r1])].copy())
                shards = [None] * world
                dist.all_gather_object(shards, (r0, r1, int(len(blk[1]))))
                ebase = engine.gather_layout(P, shards)
                blocks = [None] * world
                dist.all_gather_object(blocks, blk)
                g_rp = np.concatenate([b[0] for b in blocks])
                g_cols = np.zeros(int(ebase[-1]), np.uint16)
                g_vals = np.zeros(int(ebase[-1]), np.float32)
                for r, b in enumerate(blocks):
                    g_cols[ebase[r]:ebase[r + 1]] = b[1]
                    g_vals[ebase[r]:ebase[r + 1]] = b[2]
                # canonical entry offsets from the gathered row pointers
                g_eo = np.zeros(P + 1, np.int64)
                for p in range(P):
                    g_eo[p + 1] = g_eo[p] + g_rp[f.rp_off[p + 1] - 1]
                f.import_csr(g_rp, g_eo, g_cols, g_vals)
                rounds.append((list(map(int, bounds)), g_rp, g_eo, g_cols, g_vals))
            q.put((rank, rounds))
        finally:
            f.close()
    finally:
        dist.destroy_process_group()


def test_sharded_relaxation_matches_single_process():
    import orc
    world = 3
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_relax_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    fam = _family()
    lens = [len(s) for s in fam]
    P = len(fam) * (len(fam) - 1) // 2
    rp, cols, vals, _ = _store(fam, 0, 0, P)
    L1, ro, _ = orc.store_view(lens, np.arange(P), rp, np.zeros(P + 1, np.int64))
    blocks, e = [], 0
    for p in range(P):
        r = rp[ro[p]:ro[p] + L1[p] + 2]
        blocks.append((r.astype(np.int32), cols[e:e + r[-1]].astype(np.int32), vals[e:e + r[-1]]))
        e += r[-1]
    # the checker: the oracle's single-process rounds
    want = []
    for _ in range(ROUNDS):
        blocks = orc.relax(lens, blocks)
        want.append(blocks)
    for rank, rounds in got:
        assert len(rounds) == ROUNDS
        for it, (bounds, g_rp, g_eo, g_cols, g_vals) in enumerate(rounds):
            assert bounds[0] == 0 and bounds[-1] == P and sorted(bounds) == bounds
            assert sum(bounds[r + 1] > bounds[r] for r in range(world)) >= 2  # the work is really split
            for p in range(P):
                r = g_rp[ro[p]:ro[p] + L1[p] + 2]
                c = g_cols[g_eo[p]:g_eo[p + 1]].astype(np.int32)
                v = g_vals[g_eo[p]:g_eo[p + 1]]
                ref = want[it][p]
                assert np.array_equal(r, ref[0]) and np.array_equal(c, ref[1]) and np.array_equal(v, ref[2]), (it, p)


def test_relax_shard_plan_balance():
    """Ranges tile the pairs in order; each range's estimated work is within
    one pair of the mean (the estimate is recomputed here in numpy)."""
    from mlprobs_amd import engine
    rng = np.random.default_rng(9)
    n = 40
    lens = rng.integers(30, 300, size=n).astype(np.int32)
    P = n * (n - 1) // 2
    nnz = rng.integers(0, 4000, size=P).astype(np.int64)
    nnz[rng.random(P) < 0.2] = 0
    M = np.zeros((n, n))
    k = 0
    for a in range(n):
        for b in range(a + 1, n):
            M[a, b] = M[b, a] = nnz[k]
            k += 1
    est = (M / lens[None, :]) @ M
    cost = np.array([est[a, b] for a in range(n) for b in range(a + 1, n)]) + (n - 2) * nnz
    for R in (1, 2, 5, 8):
        b = engine.relax_shard_plan(lens, nnz, R)
        assert b[0] == 0 and b[-1] == P and all(b[r] <= b[r + 1] for r in range(R))
        loads = [cost[b[r]:b[r + 1]].sum() for r in range(R)]
        assert max(loads) <= cost.sum() / R + cost.max() * 1.0001


def test_bench_two_ranks_dry_run():
    """bench.py's N-rank path (per-rank records, all-gather timing and bytes,
    consistency rounds with their gathers) run as torchrun would on GPUs, on
    host contexts over gloo (--host): the JSON line carries the multi-rank
    fields, both ranks hold the same store after the posterior stage and each
    round, and that store is the single-process one (the library's host
    context, itself checked against the oracle above)."""
    import hashlib
    import json
    import subprocess
    from mlprobs_amd import synth
    from mlprobs_amd.engine import Family
    port = _free_port()
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2', '--master-addr',
           '127.0.0.1', '--master-port', str(port), os.path.join(ROOT, 'bench.py'), '--gpus', '2', '--host',
           '--nseq', '10', '--len', '40', '--steps', '1', '--warmup', '0', '--no-cpu', '--no-e2e', '--no-qp',
           '--no-shards', '--relax', '2']
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd='/tmp')
    assert r.returncode == 0, r.stderr[-3000:]
    last = r.stdout.strip().splitlines()[-1]
    assert len(last) < 10000
    d = json.loads(last)
    assert d['n_gpus'] == 2 and len(d['ranks']) == 2
    assert d['gather_ms'] > 0 and d['gather_GBps'] > 0
    assert all(x['gather_bytes_in'] > 0 and x['pairs'] > 0 for x in d['ranks'])
    assert sum(x['pairs'] for x in d['ranks']) == 45
    assert d['relax']['rounds'] == 2 and len(d['relax']['per_round'][0]['ranks']) == 2
    assert d['ranks_identical']

    def hsh(f):
        h = hashlib.sha256()
        for a in f.export():
            h.update(np.ascontiguousarray(a).tobytes())
        return h.hexdigest()

    seqs = [s for _, s in synth.family(10, 40, 0.7, seed=11)]
    f = Family(seqs, host=True)
    try:
        f.posteriors(0, DELTA)
        # the line carries each hash's first 16 hex digits
        assert d['ranks'][0]['store_hash'] == hsh(f)[:16]
        for rr in d['relax']['per_round']:
            f.relax(1)
            assert rr['ranks'][0]['store_hash'] == hsh(f)[:16]
    finally:
        f.close()
