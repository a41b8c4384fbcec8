"""Host stages of the c_p_np_aln drop-in (mlprobs_amd/cli/msa_host.cpp) on
the CPU: the CPU oracle supplies what the GPU computes in the real binary
(family test, posteriors, distances, consistency), tests/native/host_driver
runs the guide tree, progressive alignment and refinement, and the MFA must
equal the reference CLI's single-thread output byte for byte
(tests/golden/cli/*, made by tests/golden/gen_golden.py).
"""
import os
import struct
import subprocess
import sys

import numpy as np
import pytest

import orc
from goldens import GOLDEN
from mlprobs_amd import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, 'mlprobs_amd', 'cli')


@pytest.fixture(scope='module')
def driver(tmp_path_factory):
    out = str(tmp_path_factory.mktemp('drv') / 'host_driver')
    subprocess.check_call(['g++', '-O2', '-std=c++17', '-ffp-contract=off', '-pthread', '-I', CLI,
                           os.path.join(ROOT, 'tests', 'native', 'host_driver.cpp'),
                           os.path.join(CLI, 'msa_host.cpp'), os.path.join(CLI, 'np_host.cpp'),
                           os.path.join(CLI, 'pool.cpp'), '-o', out])
    return out


def _family_inputs(seqs, consistency, np_mode=False):
    """What the GPU computes in c_p_np_aln -p 0 (np_mode: -p 1), from the oracle."""
    m0 = orc.model(0.132548)
    vm, ident, delta = orc.model_adjustment(m0, seqs)
    pid, vpid = vm % 10, vm // 10
    m = orc.model(delta)
    n = len(seqs)
    D = np.zeros((n, n), np.float32)
    csrs = []
    for a in range(n):
        for b in range(a + 1, n):
            post = orc.pair_posterior(m, seqs[a], seqs[b], pid | (orc.NPDO if np_mode else 0))
            rp, cols, vals = orc.sparsify(len(seqs[a]), len(seqs[b]), post)
            if np_mode:  # ArrangePosteriorProbs: score / #B (CPNP/MSA.cpp:1744-1753)
                sc, path = orc.mea(len(seqs[a]), len(seqs[b]), post, with_path=True)
                D[a, b] = D[b, a] = np.float32(sc) / np.float32(path.count('B'))
            else:
                sc = orc.mea(len(seqs[a]), len(seqs[b]), post)
                D[a, b] = D[b, a] = np.float32(1) - np.float32(sc) / np.float32(min(len(seqs[a]), len(seqs[b])))
            csrs.append((rp.astype(np.int32), cols.astype(np.int32), vals.astype(np.float32)))
    lens = [len(s) for s in seqs]
    for _ in range(consistency):
        csrs = [(r.astype(np.int32), c.astype(np.int32), v.astype(np.float32)) for r, c, v in orc.relax(lens, csrs)]
    return pid, vpid, D, csrs


def _write(path, headers, seqs, pid, vpid, refinement, D, csrs, flags=0):
    with open(path, 'wb') as fh:
        fh.write(struct.pack('<5i', len(seqs), pid, vpid, refinement, flags))
        for h, s in zip(headers, seqs):
            hb = h.encode()
            fh.write(struct.pack('<i', len(hb)) + hb + struct.pack('<i', len(s)) + s.encode())
        fh.write(D.astype('<f4').tobytes())
        fh.write(np.concatenate([r for r, _, _ in csrs]).astype('<i4').tobytes())
        eo = np.zeros(len(csrs) + 1, np.int64)
        eo[1:] = np.cumsum([len(c) for _, c, _ in csrs])
        fh.write(eo.astype('<i8').tobytes())
        fh.write(np.concatenate([c for _, c, _ in csrs] + [np.zeros(0, np.int32)]).astype('<u2').tobytes())
        fh.write(np.concatenate([v for _, _, v in csrs] + [np.zeros(0, np.float32)]).astype('<f4').tobytes())


@pytest.mark.parametrize('name', ['div12', 'sim8', 'bb11028'])
@pytest.mark.parametrize('variant', ['p_0_c_0_ir_0', 'p_0'])
def test_progressive_vs_reference_cli(driver, tmp_path, name, variant):
    fam = synth.read_fasta(os.path.join(GOLDEN, 'cli', f'{name}.fa'))
    headers = [h for h, _ in fam]
    seqs = [s for _, s in fam]
    consistency, refinement = (0, 0) if variant.endswith('c_0_ir_0') else (2, 100)
    pid, vpid, D, csrs = _family_inputs(seqs, consistency)
    inp = str(tmp_path / 'in.bin')
    _write(inp, headers, seqs, pid, vpid, refinement, D, csrs)
    got = subprocess.run([driver, inp], capture_output=True, check=True).stdout.decode()
    with open(os.path.join(GOLDEN, 'cli', f'{name}_{variant}.out')) as fh:
        ref = fh.read()
    assert got == ref


NP_TIME = '1700000000'  # the clock of tests/golden/np/*.p_1.out (tests/golden/gen_np.py)
# the CPU suite takes the CLI goldens and a few real families; the drop-in
# binary runs every family of tests/golden/np on the GPU (test_cli_gpu.py)
NP_FAMILIES = ['div12', 'sim8', 'bb11028', 'bali3_BB11001', 'ox_104s10', 'oxx____8t2', 'sabre_sup_017']


def _np_family(name):
    sub = 'cli' if name in ('div12', 'sim8', 'bb11028') else 'real'
    return synth.read_fasta(os.path.join(GOLDEN, sub, f'{name}.fa'))


@pytest.mark.parametrize('name', NP_FAMILIES)
@pytest.mark.parametrize('variant', ['p_1_ir_0', 'p_1'])
def test_nonprogressive_vs_reference_cli(driver, tmp_path, name, variant):
    """-p 1 host stages (np_host.cpp: alignment graph, FindSimilar +
    DoRefinement) from the oracle's npdoAlign posteriors, distances and two
    consistency rounds, against the reference CLI byte for byte (-p 1 with
    the fixed clock of the golden run)."""
    fam = _np_family(name)
    headers = [h for h, _ in fam]
    seqs = [s for _, s in fam]
    pid, vpid, D, csrs = _family_inputs(seqs, 2, np_mode=True)
    inp = str(tmp_path / 'in.bin')
    _write(inp, headers, seqs, pid, vpid, 0 if variant.endswith('ir_0') else 100, D, csrs, flags=2)
    got = subprocess.run([driver, inp], capture_output=True, check=True,
                         env=dict(os.environ, MLP_SRAND_TIME=NP_TIME)).stdout.decode()
    with open(os.path.join(GOLDEN, 'np', f'{name}.{variant}.out')) as fh:
        ref = fh.read()
    assert got == ref
