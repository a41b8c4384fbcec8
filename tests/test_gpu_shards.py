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
    """MLP_FORCE_PEER=1: the all-gather's copies take the hipMemcpyPeerAsync
    branch even between shards of one device (the xGMI path of a real
    multi-GPU box)."""
    monkeypatch.setenv('MLP_FORCE_PEER', '1')
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
