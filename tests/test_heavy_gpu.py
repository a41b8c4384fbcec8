"""The families the drop-ins actually send to the GPU: 12 TEST/ox + TEST/sabre
families above the host-path bound (4.6e6 .. 9.6e7 pair-cells, 46% of C5's
pair-cells; tests/golden/pipeline_heavy, made by
`tests/golden/gen_pipeline.py --heavy` from the reference's utils/*.py
driving the reference CLIs built from source, single-threaded, fixed clock).

Default dispatch throughout (no MLP_HOST_MAX_CELLS override): the pipeline
driver must route the family's base MSA to the device by itself (trace
`device_runs` > 0), reproduce every stage and the final bytes; the two
drop-in CLIs must reproduce the reference CLIs' own outputs (c_p_np_aln -p 0,
-p 1 with refinement under the fixed clock, quickprobs) byte for byte.  The
CPU suite runs the same fixtures through the host path for the smallest
families (tests/test_pipeline.py style), so a failure here isolates the
device path."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(ROOT, 'tests', 'golden', 'pipeline_heavy')
CLI = os.path.join(ROOT, 'mlprobs_amd', 'cli')
FIXED_TIME = '1700000000'
ENV = dict(os.environ, MLP_SRAND_TIME=FIXED_TIME)
ENV.pop('MLP_HOST_MAX_CELLS', None)


def manifest():
    with open(os.path.join(FIX, 'manifest.json')) as fh:
        return json.load(fh)['families']


def tags():
    return [f['tag'] for f in manifest()]


def load(tag):
    with open(os.path.join(FIX, f'{tag}.json')) as fh:
        return json.load(fh)


def run_pipeline(tag, tmp, env):
    from test_pipeline import check_trace
    rec = load(tag)
    out, trace = os.path.join(tmp, 'o.msa'), os.path.join(tmp, 't.json')
    r = subprocess.run([os.path.join(CLI, 'mlprobs'), '-q', '--trace', trace, os.path.join(FIX, f'{tag}.fa'), out],
                       capture_output=True, timeout=900, env=env)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    with open(trace) as fh:
        tr = json.load(fh)
    check_trace(rec, tr, tag)
    with open(out, encoding='latin-1') as fh:
        assert fh.read() == rec['final'], tag
    return tr


@pytest.mark.gpu
@pytest.mark.parametrize('tag', tags())
def test_heavy_pipeline_default_dispatch(tag, tmp_path):
    tr = run_pipeline(tag, str(tmp_path), ENV)
    assert tr['device_runs'] > 0, (tag, tr['device_runs'], tr['host_runs'])


@pytest.mark.gpu
@pytest.mark.parametrize('mode', ['p_0', 'p_1', 'qp'])
@pytest.mark.parametrize('tag', tags())
def test_heavy_cli_default_dispatch(tag, mode):
    rec = load(tag)
    rc, want = rec['reference_cli'][mode]
    fa = os.path.join(FIX, f'{tag}.fa')
    cmd = ([os.path.join(CLI, 'quickprobs'), fa] if mode == 'qp' else
           [os.path.join(CLI, 'c_p_np_aln'), '-p', mode[-1], fa])
    r = subprocess.run(cmd, capture_output=True, timeout=900, env=ENV)
    assert r.returncode == rc, r.stderr.decode()[-2000:]
    assert r.stdout.decode('latin-1') == want, (tag, mode)


def _smallest(k):
    return [f['tag'] for f in sorted(manifest(), key=lambda f: f['cells'])[:k]]


@pytest.mark.parametrize('tag', _smallest(2))
def test_heavy_pipeline_host_path(tag, tmp_path):
    """The same fixtures on the CPU (host context forced for every size), for
    the two smallest heavy families: pins the fixtures themselves in the CPU
    suite and separates a device-path failure from a host-stage one."""
    run_pipeline(tag, str(tmp_path), dict(ENV, MLP_HOST_MAX_CELLS='1e12', MLP_HOST_THREADS='4'))
