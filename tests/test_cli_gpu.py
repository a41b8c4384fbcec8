"""The c_p_np_aln drop-in binary (mlprobs_amd/cli) on the GPU against the
reference CLI's single-thread outputs (tests/golden/cli)."""
import os
import subprocess

import pytest

from goldens import GOLDEN

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, 'mlprobs_amd', 'cli', 'c_p_np_aln')

pytestmark = pytest.mark.gpu


def _run(*args):
    return subprocess.run([BIN, *args], capture_output=True, text=True, timeout=300)


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


def test_cli_errors():
    assert _run('-version').returncode == 1
    assert _run('-zz').returncode == 1
    assert _run('-p', '2', 'x.fa').returncode == 1
    r = _run('-p', '1', os.path.join(GOLDEN, 'cli', 'sim8.fa'))
    assert r.returncode != 0
