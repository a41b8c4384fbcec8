"""The MEA recurrence on host SIMD lanes (mlprobs_amd/cli/msa_host.cpp
mea_path_simd, used by both drop-ins' progressive alignment and refinement)
against the serial recurrence (ChooseBestOfThree, CPNP/ScoreType.h:347-366;
QuickProbs' computeAlignment is the same): path and score bit for bit on
3000 random shapes per lane count, including quantised posteriors whose
ties exercise every branch of the compare order."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, 'mlprobs_amd', 'cli')


def _cpu_has(flag):
    try:
        with open('/proc/cpuinfo') as fh:
            for line in fh:
                if line.startswith('flags'):
                    return flag in line.split()
    except OSError:
        pass
    return False


@pytest.fixture(scope='module')
def checker(tmp_path_factory):
    out = str(tmp_path_factory.mktemp('mea') / 'mea_check')
    subprocess.check_call(['g++', '-O2', '-std=c++17', '-ffp-contract=off', '-pthread', '-I', CLI,
                           os.path.join(ROOT, 'tests', 'native', 'mea_check.cpp'),
                           os.path.join(CLI, 'msa_host.cpp'), os.path.join(CLI, 'pool.cpp'), '-o', out])
    return out


@pytest.mark.parametrize('lanes,flag,threads', [(8, 'avx2', 1), (16, 'avx512bw', 1), (16, 'avx512bw', 4)])
def test_mea_simd_matches_serial(checker, lanes, flag, threads):
    """threads > 1: the 16-lane strips pipelined over host threads."""
    if not _cpu_has(flag):
        pytest.skip(f'no {flag} on this CPU')
    env = dict(os.environ, MLP_HOST_THREADS=str(threads), MLP_MEA_THREAD_MIN='1' if threads > 1 else '0')
    r = subprocess.run([checker, str(lanes)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith('ok 3000')
