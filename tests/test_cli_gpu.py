"""The c_p_np_aln drop-in binary (mlprobs_amd/cli) on the GPU against the
reference CLI's single-thread outputs (tests/golden/cli).  MLP_HOST_MAX_CELLS=0
keeps every family on the GPU path (small families would otherwise take the
host path, which tests/test_cli_hostpath.py covers in the CPU suite)."""
import os
import subprocess

import pytest

from goldens import GOLDEN

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, 'mlprobs_amd', 'cli', 'c_p_np_aln')

pytestmark = pytest.mark.gpu
ENV = dict(os.environ, MLP_HOST_MAX_CELLS='0')  # every CLI process of this module: the GPU path


def _run(*args):
    return subprocess.run([BIN, *args], capture_output=True, text=True, timeout=300, env=ENV)


@pytest.mark.parametrize('name', ['bb11028', 'div12', 'sim8'])
def test_cli_features(name):
    r = _run('-G', os.path.join(GOLDEN, 'cli', f'{name}.fa'))
    assert r.returncode == 0 and r.stderr == '', r.stderr
    with open(os.path.join(GOLDEN, 'cli', f'{name}_G.out')) as fh:
        assert r.stdout == fh.read()


@pytest.mark.parametrize('name', ['bb11028', 'div12', 'sim8'])
@pytest.mark.parametrize('flags,suffix', [((), 'p_0'), (('-c', '0', '-ir', '0'), 'p_0_c_0_ir_0')])
def test_cli_progressive(name, flags, suffix):
    r = _run('-p', '0', *flags, os.path.join(GOLDEN, 'cli', f'{name}.fa'))
    assert r.returncode == 0 and r.stderr == '', r.stderr
    with open(os.path.join(GOLDEN, 'cli', f'{name}_{suffix}.out')) as fh:
        assert r.stdout == fh.read()


@pytest.mark.parametrize('name', ['bb11028', 'div12', 'sim8'])
@pytest.mark.parametrize('flags,suffix', [((), 'p_0'), (('-p', '1'), 'p_1'), (('-p', '1', '-ir', '0'), 'p_1_ir_0')])
@pytest.mark.parametrize('mea', ['host', 'device', 'device-gives-up'])
def test_cli_profile_posterior_on_gpu(name, flags, suffix, mea):
    """Every progressive merge and refinement pass through the GPU's
    BuildPosterior (MLP_PROFILE_GPU_MIN=1: no host fallback for small
    profile pairs), its MEA on the host or on the device
    (MLP_MEA_GPU_MIN=0: mlp_profile_mea for every merge): still the
    reference's bytes."""
    env = dict(ENV, MLP_PROFILE_GPU_MIN='1', MLP_SRAND_TIME='1700000000')
    if mea.startswith('device'):
        env['MLP_MEA_GPU_MIN'] = '0'
        if mea == 'device-gives-up':   # every device MEA may give up: the host fallback
            env['MLP_TEST_MEA_SPINS'] = '0'
    else:
        env['MLP_MEA_GPU_MIN'] = str(1 << 40)
    r = subprocess.run([BIN, *(flags or ('-p', '0')), os.path.join(GOLDEN, 'cli', f'{name}.fa')], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0 and r.stderr == '', r.stderr
    ref = os.path.join(GOLDEN, 'cli', f'{name}_{suffix}.out') if suffix == 'p_0' else \
        os.path.join(GOLDEN, 'np', f'{name}.{suffix}.out')
    with open(ref) as fh:
        assert r.stdout == fh.read()


def test_cli_errors():
    assert _run('-version').returncode == 1
    assert _run('-zz').returncode == 1
    assert _run('-p', '2', 'x.fa').returncode == 1


# ---- the non-progressive strategy (-p 1, npdoAlign) against the reference
# CLI (tests/golden/np, tests/golden/gen_np.py): -ir 0 (alignment graph) and
# the default refinement under the golden run's fixed clock
NP = os.path.join(GOLDEN, 'np')
_NP = sorted(f[:-len('.p_1.out')] for f in os.listdir(NP) if f.endswith('.p_1.out')) if os.path.isdir(NP) else []
NP_TIME = '1700000000'


def _fasta_of(name):
    for sub in ('cli', 'real', 'edge'):
        fa = os.path.join(GOLDEN, sub, f'{name}.fa')
        if os.path.exists(fa):
            return fa
    raise FileNotFoundError(name)


@pytest.mark.parametrize('name', _NP)
def test_cli_nonprogressive(name):
    fa = _fasta_of(name)
    for tag, args in (('p_1_ir_0', ['-p', '1', '-ir', '0']), ('p_1', ['-p', '1'])):
        r = subprocess.run([BIN, *args, fa], capture_output=True, timeout=300,
                           env=dict(ENV, MLP_SRAND_TIME=NP_TIME))
        assert r.returncode == 0 and r.stderr == b'', (tag, r.stderr)
        with open(os.path.join(NP, f'{name}.{tag}.out'), 'rb') as fh:
            assert r.stdout == fh.read(), (name, tag)


# ---- the quickprobs drop-in (QuickProbs 2 realigner) against the reference
# QuickProbs CLI built from its sources (tests/golden/cli/qp_*.out)
QP_BIN = os.path.join(ROOT, 'mlprobs_amd', 'cli', 'quickprobs')


@pytest.mark.parametrize('name,args', [('bb11028', []), ('bb11028', ['-c', '0']), ('bb11028', ['-c', '1', '-r', '5']),
                                       ('div12', []), ('div12', ['-c', '0']), ('sim8', []),
                                       ('sim8', ['-c', '3', '-r', '50']), ('qp_div60', []), ('qp_big210', []),
                                       ('div12', ['hostmea']), ('qp_div60', ['hostmea']),
                                       ('qp_big210', ['hostmea'])])
def test_quickprobs_cli(name, args):
    env = ENV   # every MEA on the device (mlp_profile_mea, the default)
    if args == ['hostmea']:  # every MEA on the host
        args, env = [], dict(ENV, MLP_MEA_DEVICE='0')
    r = subprocess.run([QP_BIN, *args, os.path.join(GOLDEN, 'cli', f'{name}.fa')], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0 and r.stderr == '', r.stderr
    tag = 'qp_' + name.replace('qp_', '') + ''.join('_' + a.strip('-') for a in args)
    with open(os.path.join(GOLDEN, 'cli', f'{tag}.out')) as fh:
        assert r.stdout == fh.read()


def test_quickprobs_cli_edges(tmp_path):
    r = subprocess.run([QP_BIN], capture_output=True, text=True, timeout=60, env=ENV)
    assert r.returncode == 0 and r.stdout.startswith('Usage:')        # no input: usage (main.cpp:31-37)
    bad = tmp_path / 'bad.fa'
    bad.write_text('>a\nMK1V\n>b\nMKV\n')
    r = subprocess.run([QP_BIN, str(bad)], capture_output=True, text=True, timeout=60, env=ENV)
    assert r.returncode == 255 and 'illegal sequence character:1' in r.stdout
    one = tmp_path / 'one.fa'
    one.write_text('>only one\nmkvlaa\nGG\n')
    r = subprocess.run([QP_BIN, '-o', str(tmp_path / 'o.fa'), str(one)], capture_output=True, text=True, timeout=60, env=ENV)
    assert r.returncode == 0 and (tmp_path / 'o.fa').read_text() == '>only one\nMKVLAAGG\n'


# ---- both drop-ins on real benchmark families (the reference's own TEST
# inputs, tests/golden/real, made by tests/golden/gen_real.py from the
# reference CLIs built from source)
REAL = os.path.join(GOLDEN, 'real')
_REAL = sorted(f[:-3] for f in os.listdir(REAL) if f.endswith('.fa')) if os.path.isdir(REAL) else []


@pytest.mark.parametrize('name', _REAL)
def test_real_families(name):
    fa = os.path.join(REAL, f'{name}.fa')
    for tag, cmd in (('G', [BIN, '-G', fa]), ('p_0', [BIN, '-p', '0', fa]), ('qp', [QP_BIN, fa])):
        if not os.path.exists(os.path.join(REAL, f'{name}.{tag}.out')):
            continue  # the larger oxxL_ families are quickprobs-only
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=ENV)
        assert r.returncode == 0 and r.stderr == '', (tag, r.stderr)
        with open(os.path.join(REAL, f'{name}.{tag}.out')) as fh:
            assert r.stdout == fh.read(), (name, tag)


EDGE = os.path.join(GOLDEN, 'edge')
_EDGE = sorted(f[:-3] for f in os.listdir(EDGE) if f.endswith('.fa')) if os.path.isdir(EDGE) else []


@pytest.mark.parametrize('name', _EDGE)
def test_edge_families(name):
    """Two sequences, single residues, identical sequences, lower case and
    X/B/Z, CRLF line ends (tests/golden/gen_edge.py)."""
    fa = os.path.join(EDGE, f'{name}.fa')
    for tag, cmd in (('G', [BIN, '-G', fa]), ('p_0', [BIN, '-p', '0', fa]), ('qp', [QP_BIN, fa])):
        r = subprocess.run(cmd, capture_output=True, timeout=120, env=ENV)  # bytes: CR stays CR
        assert r.returncode == 0 and r.stderr == b'', (tag, r.stderr)
        with open(os.path.join(EDGE, f'{name}.{tag}.out'), 'rb') as fh:
            assert r.stdout == fh.read(), (name, tag)


# ---- BASELINE.json configurations end to end: the reference CLI's `-p 0`
# output on the bench's own synthetic families (tests/golden/config,
# tools/gen_config_goldens.sh: C2 single-threaded; C3 has more than 150
# sequences, so refinement is off and the reference's threads cannot race)
@pytest.mark.parametrize('name', ['c2_128x256_s11', 'c3_512x400_s11'])
def test_cli_config_families(name):
    out = os.path.join(GOLDEN, 'config', f'{name}.p_0.out')
    if not os.path.exists(out):
        pytest.skip('reference output not generated')
    r = _run('-p', '0', os.path.join(GOLDEN, 'config', f'{name}.fa'))
    assert r.returncode == 0 and r.stderr == '', r.stderr
    with open(out) as fh:
        assert r.stdout == fh.read()


def test_cli_config_c2_nonprogressive():
    """C2 with -p 1 (alignment graph + refinement: some 130 profile MEAs of up
    to 4263 x 7288 columns on the device) under the golden run's fixed clock:
    the reference CLI's bytes (round 5: an unmasked edge block of the device
    MEA diverged here)."""
    out = os.path.join(GOLDEN, 'config', 'c2_128x256_s11.p_1.out')
    r = subprocess.run([BIN, '-p', '1', os.path.join(GOLDEN, 'config', 'c2_128x256_s11.fa')], capture_output=True,
                       text=True, timeout=300, env=dict(ENV, MLP_SRAND_TIME=NP_TIME))
    assert r.returncode == 0 and r.stderr == '', r.stderr
    with open(out) as fh:
        assert r.stdout == fh.read()


@pytest.mark.parametrize('name', ['c2_128x256_s11', 'c3_512x400_s11'])
def test_quickprobs_config_families(name):
    """The quickprobs drop-in on the bench's C2 / C3 families: the reference
    QuickProbs CLI's output (tools/gen_config_goldens.sh)."""
    out = os.path.join(GOLDEN, 'config', f'{name}.qp.out')
    if not os.path.exists(out):
        pytest.skip('reference output not generated')
    r = subprocess.run([QP_BIN, os.path.join(GOLDEN, 'config', f'{name}.fa')], capture_output=True, text=True,
                       timeout=300, env=ENV)
    assert r.returncode == 0 and r.stderr == '', r.stderr
    with open(out) as fh:
        assert r.stdout == fh.read()


@pytest.mark.parametrize('name', ['qp_div60', 'qp_big210'])
def test_quickprobs_device_mea_gives_up(name):
    """A device MEA strip that gives up waiting for the one above
    (MLP_TEST_MEA_SPINS=0: at the first poll that finds it not ready) returns
    MLP_ERR_STATE and the drop-in computes that MEA on the host: still the
    reference's bytes, nothing on stderr."""
    env = dict(ENV, MLP_TEST_MEA_SPINS='0', MLP_MEA_GPU_MIN='0')
    r = subprocess.run([QP_BIN, os.path.join(GOLDEN, 'cli', f'{name}.fa')], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0 and r.stderr == '', r.stderr
    with open(os.path.join(GOLDEN, 'cli', f'{name}.out' if name.startswith('qp_') else f'qp_{name}.out')) as fh:
        assert r.stdout == fh.read()
