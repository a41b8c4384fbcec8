"""In-process multi-GPU path of the C ABI (mlp_ctx_create_mask /
mlp_set_shards): k shards (child contexts) each compute a contiguous pair
range, their sparse sets are gathered into the parent's canonical store, and
every consistency round relaxes MAC-balanced output ranges on the shards from
a copy of the whole store.  On a one-GPU box the shards are virtual (they
share the device) and the gather is a device copy; the store, distances and
every relaxation round must equal the unsharded run bit for bit (SURVEY.md
section 8b: results independent of the GPU count).  Real N > 1 devices are
unmeasured here."""
import numpy as np
import pytest

from mlprobs_amd import synth
from mlprobs_amd.engine import PID_QP, Family

pytestmark = pytest.mark.gpu


def _same(a, b, what):
    for x, y, name in zip(a.export(), b.export(), ('row_ptr', 'ent_off', 'cols', 'vals')):
        np.testing.assert_array_equal(x, y, err_msg=f'{what} {name}')
    for x, y in zip(a.results(), b.results()):
        np.testing.assert_array_equal(x, y, err_msg=f'{what} per-pair results')


@pytest.mark.parametrize('k', [2, 4])
@pytest.mark.parametrize('pid', [0, 2])
def test_virtual_shards_posteriors_and_relax(k, pid):
    seqs = [s for _, s in synth.family(48, 160, 0.7, seed=91)]
    one = Family(seqs)
    many = Family(seqs, shards=k)
    one.posteriors(pid, 0.132548)
    many.posteriors(pid, 0.132548)
    _same(one, many, f'k={k} posteriors')
    for it in range(2):
        one.relax(1)
        many.relax(1)
        _same(one, many, f'k={k} relax round {it + 1}')
    many.relax(2)  # several rounds in one call
    one.relax(2)
    _same(one, many, f'k={k} relax x2')
    one.close()
    many.close()


@pytest.mark.parametrize('k', [3])
def test_virtual_shards_quickprobs(k):
    seqs = [s for _, s in synth.family(30, 140, 0.6, seed=92)]
    rng = np.random.default_rng(3)
    w = rng.uniform(1, 20, len(seqs)).astype(np.float32)
    seld = rng.integers(2, len(seqs), (len(seqs), len(seqs))).astype(np.float32)
    seld = np.minimum(seld, seld.T)
    np.fill_diagonal(seld, 0)
    one = Family(seqs)
    many = Family(seqs, shards=k)
    for f in (one, many):
        f.posteriors(PID_QP, 0.0)
        f.relax_qp(2, w, seld, 8.0)
    _same(one, many, 'quickprobs')
    one.close()
    many.close()


@pytest.mark.parametrize('k', [2, 8])
def test_virtual_shards_forced_peer_copies(k, monkeypatch):
    """MLP_TEST_FORCE_PEER=1: the all-gather's copies take the hipMemcpyPeerAsync
    branch even between shards of one device (the xGMI path of a real
    multi-GPU box)."""
    monkeypatch.setenv('MLP_TEST_FORCE_PEER', '1')
    seqs = [s for _, s in synth.family(40, 150, 0.7, seed=93)]
    one = Family(seqs)
    many = Family(seqs, shards=k)
    one.posteriors(0, 0.132548)
    many.posteriors(0, 0.132548)
    _same(one, many, f'k={k} peer posteriors')
    one.relax(2)
    many.relax(2)
    _same(one, many, f'k={k} peer relax x2')
    one.close()
    many.close()


def test_virtual_shards_imported_store():
    """A store the shards never saw (mlp_csr_import) is sent out before the
    first sharded round, then all-gathered after each."""
    seqs = [s for _, s in synth.family(36, 140, 0.7, seed=94)]
    one = Family(seqs)
    one.posteriors(0, 0.132548)
    many = Family(seqs, shards=3)
    many.import_csr(*one.export())
    one.relax(1)
    many.relax(1)
    for x, y in zip(one.export(), many.export()):
        np.testing.assert_array_equal(x, y)
    one.close()
    many.close()


_RCCL_CHILD = r'''
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from mlprobs_amd import synth
from mlprobs_amd.engine import Family

def store(f):
    return [a.copy() for a in f.export()] + [a.copy() for a in f.results()]

def same(a, b, what):
    for k, (x, y) in enumerate(zip(a, b)):
        assert np.array_equal(x, y), (what, k)

seqs = [s for _, s in synth.family(40, 150, 0.7, seed=93)]
ref = Family(seqs)
ref.posteriors(0, 0.132548)
s_post = store(ref)
ref.relax(1)
s_relax = store(ref)
ref.close()
f = Family(seqs)
f.comm_init(Family.unique_id(), 1, 0)
f.profile(True)
f.posteriors(0, 0.132548)
f.allgather()
assert f.kernel_times()['allgather']['launches'] > 0, 'the grouped body did not run'
same(store(f), s_post, 'posteriors after the RCCL all-gather')
# a rank's relaxation round followed by its all-gather, as mlp_relax does
# with several ranks
f.relax(1)
f.allgather()
same(store(f), s_relax, 'relax round after the RCCL all-gather')
f.close()
print('rccl allgather ok')
'''


def test_rccl_allgather_grouped_body_one_rank():
    """The one-process-per-GPU path's RCCL all-gather (mlp_comm_init +
    mlp_allgather's grouped broadcasts, per-rank entry placement, scalar
    exchange, ent_off rebuild) at one rank, forced past the one-rank early
    return (MLP_TEST_ALLGATHER_FORCE=1): the store, distances and MEA scores after
    the gather equal the context's own, after the posterior stage and after a
    relaxation round.  In a child process: the hook is read once per
    process."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, '-c', _RCCL_CHILD, root], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, MLP_TEST_ALLGATHER_FORCE='1'))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert 'rccl allgather ok' in r.stdout


def test_relax_range_matches_full_round():
    """mlp_relax_range on the device: each output range's block equals the
    same pairs of a full round, bit for bit, and the entry offsets outside the
    range are laid out as the host context lays them out."""
    seqs = [s for _, s in synth.family(36, 150, 0.7, seed=94)]
    full = Family(seqs)
    full.posteriors(0, 0.132548)
    base = [a.copy() for a in full.export()]
    full.relax(1)
    rp_f, eo_f, c_f, v_f = full.export()
    P = len(eo_f) - 1
    for r0, r1 in ((0, P // 3), (P // 3, P), (P // 2, P // 2 + 1)):
        part = Family(seqs)
        part.import_csr(*base)
        part.relax_range(r0, r1)
        rp, eo, c, v = part.export()
        a, b = int(part.rp_off[r0]), int(part.rp_off[r1])
        np.testing.assert_array_equal(rp[a:b], rp_f[a:b])
        np.testing.assert_array_equal(c[int(eo[r0]):int(eo[r1])], c_f[int(eo_f[r0]):int(eo_f[r1])])
        np.testing.assert_array_equal(v[int(eo[r0]):int(eo[r1])], v_f[int(eo_f[r0]):int(eo_f[r1])])
        # the whole entry-offset layout as the host context leaves it (0
        # before r0, the range's total after r1)
        host = Family(seqs, host=True)
        host.import_csr(*base)
        host.relax_range(r0, r1)
        np.testing.assert_array_equal(eo, host.export()[1])
        host.close()
        part.close()
    full.close()


def test_virtual_shards_default_budget():
    """Shards sharing a device on the library's default scratch budget (no
    set_scratch): the budget they split leaves room for each shard's store
    copy and gather buffers; store, distances and a relaxation round equal the
    one-context run."""
    seqs = [s for _, s in synth.family(40, 180, 0.7, seed=61)]
    one = Family(seqs)
    one.posteriors(0, 0.132548)
    many = Family(seqs, shards=4)
    many.posteriors(0, 0.132548)
    _same(one, many, 'default budget posteriors')
    one.relax(1)
    many.relax(1)
    _same(one, many, 'default budget relax round')
    one.close()
    many.close()


def test_device_pool_reuse_across_contexts():
    """The process's device pool (mlp_pool_info / mlp_pool_trim): a closed
    context's batch scratch and store go back to the pool, the next context
    (a new family, then 4 virtual shards over it) is carved from the same
    blocks, and its results equal a run after
    the pool was trimmed (fresh allocations)."""
    from mlprobs_amd import engine
    seqs = [s for _, s in synth.family(40, 150, 0.7, seed=95)]
    a = Family(seqs)
    a.set_scratch(2 << 30)
    a.posteriors(0, 0.132548)
    a.relax(1)
    ref = [x.copy() for x in a.export()] + [x.copy() for x in a.results()]
    a.close()
    held, free = engine.pool_info(0)
    assert held > 0 and free == held           # everything back in the pool, nothing returned to the driver
    b = Family(seqs, shards=4)
    b.posteriors(0, 0.132548)
    b.relax(1)
    got = list(b.export()) + list(b.results())
    held2, free2 = engine.pool_info(0)
    b.close()
    assert engine.pool_info(0)[0] <= 32 << 30  # the last close shrinks the pool (MLP_POOL_KEEP_GB)
    assert held2 >= held and free2 < held      # carved from the same blocks (and more if they needed it)
    for x, y in zip(ref, got):
        np.testing.assert_array_equal(x, y)
    engine.pool_trim(0)
    assert engine.pool_info(0) == (0, 0)
    c = Family(seqs)
    c.posteriors(0, 0.132548)
    c.relax(1)
    for x, y in zip(ref, list(c.export()) + list(c.results())):
        np.testing.assert_array_equal(x, y)
    c.close()
