"""The local-model chain totals three ways (CPNP/ProbabilisticModel.h:435-450:
one serial, non-associative LOG_ADD chain per pair): one wave per pair with
the running-maximum skip bound (MLP_TEST_TOT_FOLDBOUND=0), the same with the
folded chunk-maximum bound (=1), and one pair per lane after a listing pass
into the local backward array between the two sweeps (MLP_TEST_TOT_LANEFOLD=1,
the default above the CLIs' 48 GB scratch), also with every pair sent
through the lane fold's repair pass
(MLP_TEST_TOT_FORCE_REPAIR).  All are exact, so the sparse store, distances and
MEA scores must be bit-identical, at pid 0, 1 and 2 (the local model alone:
no side stream) on similar and divergent families, and with several batches
and the PF posterior in the Zm slots (small scratch budget) as well.  The
one-wave totals run after both sweeps (MLP_TEST_TOT_BESIDE=0, the reference run
here) or with their forward chains on a second stream beside the backward
sweeps (=1, and =2 the default: the partition function joined before the
merge only).  Several batches also run with the next batch launched before
the last one is finished (the default) and finished first
(MLP_TEST_DEFER_FINISH=0).  Each setting runs in a child process: the switches
are read once per process."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r'''
import hashlib, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from mlprobs_amd import synth
from mlprobs_amd.engine import Family
out = []
for n, L, s, seed, pid in ((48, 300, 0.7, 31, 0), (40, 260, 0.35, 32, 0), (36, 220, 0.9, 33, 1), (6, 900, 0.6, 34, 0),
                           (30, 240, 0.6, 35, 2)):
    seqs = [q for _, q in synth.family(n, L, s, seed=seed)]
    f = Family(seqs)
    if len(sys.argv) > 2:
        f.set_scratch(int(sys.argv[2]))
    f.posteriors(pid, 0.132548)
    h = hashlib.sha256()
    for a in list(f.export()) + list(f.results()):
        h.update(np.ascontiguousarray(a).tobytes())
    out.append(h.hexdigest())
    f.close()
print(' '.join(out))
'''


def _run(lanefold, scratch=None, foldbound=1, repair=False, beside=2, defer=1):
    env = dict(os.environ, MLP_TEST_TOT_LANEFOLD=str(lanefold), MLP_TEST_TOT_FOLDBOUND=str(foldbound),
               MLP_TEST_TOT_BESIDE=str(beside), MLP_TEST_DEFER_FINISH=str(defer))
    env.pop('MLP_TEST_TOT_FORCE_REPAIR', None)
    if repair:
        env['MLP_TEST_TOT_FORCE_REPAIR'] = '1'
    args = [sys.executable, '-c', _CHILD, ROOT] + ([str(scratch)] if scratch else [])
    r = subprocess.run(args, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    return r.stdout.split()


def test_totals_bit_identical():
    ref = _run(0, foldbound=0, beside=0)
    assert _run(0, foldbound=0) == ref
    assert _run(0, beside=1) == ref
    assert _run(0) == ref
    assert _run(1) == ref
    assert _run(1, repair=True) == ref


def test_totals_bit_identical_small_scratch():
    # 1 GB: several batches, the PF posterior in the low halves of the Zm
    # slots (the lane fold's candidates in the local backward array either way)
    ref = _run(0, 1 << 30, foldbound=0, beside=0, defer=0)
    assert _run(0, 1 << 30, foldbound=0, beside=0) == ref
    assert _run(0, 1 << 30, foldbound=0) == ref
    assert _run(1, 1 << 30, defer=0) == ref
    assert _run(0, 1 << 30, beside=1) == ref
    assert _run(0, 1 << 30) == ref
    assert _run(1, 1 << 30) == ref
    assert _run(1, 1 << 30, repair=True) == ref


@pytest.mark.parametrize('lanefold', ['0', '1'])
def test_totals_timed_once_per_batch(lanefold):
    """The local totals group is one timed launch per batch whether its
    kernels run in one part or two (forward chains beside the backward sweeps
    / lane fold before it, backward chains after it): launches and cells equal
    the forward group's, so per-launch rooflines are not halved."""
    import numpy as np  # noqa: F401
    sys.path.insert(0, ROOT)
    from mlprobs_amd import synth
    from mlprobs_amd.engine import Family
    os.environ['MLP_TEST_TOT_LANEFOLD'] = lanefold
    try:
        f = Family([q for _, q in synth.family(48, 300, 0.7, seed=31)])
        f.set_scratch(1 << 30)
        f.profile(True)
        f.posteriors(0, 0.132548)
        f.synchronize()
        kt = f.kernel_times()
        f.close()
    finally:
        del os.environ['MLP_TEST_TOT_LANEFOLD']
    assert kt['forward']['launches'] > 1
    assert kt['local_totals']['launches'] == kt['forward']['launches']
    assert kt['local_totals']['cells'] == kt['forward']['cells']
    assert 0 < kt['local_totals']['ms']
