"""Host stages of the quickprobs drop-in (mlprobs_amd/cli/qp_host.cpp) on the
CPU: the CPU oracle supplies what the GPU computes in the real binary
(QuickProbs posterior stage, distances, consistency with the subtree-size
selectivity), tests/native/qp_host_driver runs the guide tree, weights,
progressive construction and column refinement, and the FASTA must equal the
reference QuickProbs CLI's output byte for byte (tests/golden/cli/qp_*.out,
oracle/_ref/quickprobs built from the reference sources, made by
tests/golden/gen_golden.py --qpcli).
"""
import os
import struct
import subprocess

import numpy as np
import pytest

import orc
from goldens import GOLDEN
from mlprobs_amd import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, 'mlprobs_amd', 'cli')

CASES = [('bb11028', []), ('bb11028', ['-c', '0']), ('bb11028', ['-c', '1', '-r', '5']), ('div12', []),
         ('div12', ['-c', '0']), ('sim8', []), ('sim8', ['-c', '3', '-r', '50']), ('qp_div60', []),
         ('qp_big210', [])]


def golden_name(name, args):
    return 'qp_' + name.replace('qp_', '') + ''.join('_' + a.strip('-') for a in args) + '.out'


@pytest.fixture(scope='module')
def qdriver(tmp_path_factory):
    out = str(tmp_path_factory.mktemp('qdrv') / 'qp_host_driver')
    subprocess.check_call(['g++', '-O2', '-std=c++17', '-ffp-contract=off', '-pthread', '-I', CLI,
                           os.path.join(ROOT, 'tests', 'native', 'qp_host_driver.cpp'),
                           os.path.join(CLI, 'qp_host.cpp'), os.path.join(CLI, 'msa_host.cpp'),
                           os.path.join(CLI, 'pool.cpp'), '-o', out])
    return out


def _opt(args, flag, default):
    return int(args[args.index(flag) + 1]) if flag in args else default


def _posteriors(seqs):
    """QuickProbs' posterior stage from the oracle: CSR with the 16-bit values
    as QuickProbs reads them, and the distance matrix."""
    m = orc.model(-1.0)
    n = len(seqs)
    D = np.zeros((n, n), np.float32)
    csrs = []
    for a in range(n):
        for b in range(a + 1, n):
            _, _, p, dist = orc.qp_pair(m, seqs[a], seqs[b])
            rp, cols, q = orc.qp_sparsify(len(seqs[a]), len(seqs[b]), p)
            D[a, b] = D[b, a] = dist
            csrs.append((rp.astype(np.int32), cols.astype(np.int32), q.astype(np.float32) / np.float32(65535)))
    return D, csrs


REAL = ['bali3_BB11001', 'bali3_BB12005', 'ox_581s18', 'oxx_588s27', 'oxx____397', 'sabre_sup_062']


@pytest.mark.parametrize('name,args', CASES + [('real/' + r, []) for r in REAL])
def test_quickprobs_host_vs_reference_cli(qdriver, tmp_path, name, args):
    """`real/...`: the reference's own benchmark families (tests/golden/real)."""
    fam = synth.read_fasta(os.path.join(GOLDEN, 'cli' if not name.startswith('real/') else '', f'{name}.fa'))
    headers = [h for h, _ in fam]
    seqs = [s for _, s in fam]
    n = len(seqs)
    D, csrs = _posteriors(seqs)
    # guide tree -> weights and subtree distances (host code under test)
    tin, tout = str(tmp_path / 't.bin'), str(tmp_path / 't.out')
    with open(tin, 'wb') as fh:
        fh.write(struct.pack('<i', n) + D.astype('<f4').tobytes())
    subprocess.check_call([qdriver, 'tree', tin, tout])
    raw = np.fromfile(tout, '<f4')
    w, seld = raw[:n], raw[n:].reshape(n, n)
    # consistency (oracle; ExtendedMSA.cpp:176-177, ConsistencyStage defaults)
    iters = _opt(args, '-c', -1)
    if iters < 0:
        iters = 1 if n > 50 else 2
    wc = np.maximum(w, np.float32(1e-6))
    lens = [len(s) for s in seqs]
    for it in range(1, iters + 1):
        cut = 1e-5 if it == iters else 0.01
        csrs = [(r.astype(np.int32), c.astype(np.int32), v.astype(np.float32))
                for r, c, v in orc.relax(lens, csrs, qp=(wc, 3.0, cut, seld, 200.0))]
    inp = str(tmp_path / 'in.bin')
    with open(inp, 'wb') as fh:
        fh.write(struct.pack('<2i', n, _opt(args, '-r', -1)))
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
    got = subprocess.run([qdriver, 'align', inp], capture_output=True, check=True).stdout.decode()
    ref_out = (os.path.join(GOLDEN, name + '.qp.out') if name.startswith('real/')
               else os.path.join(GOLDEN, 'cli', golden_name(name, args)))
    with open(ref_out) as fh:
        ref = fh.read()
    assert got == ref


@pytest.mark.parametrize('seed,L1,L2', [(1, 700, 650), (2, 129, 2100), (3, 1500, 257)])
def test_mea_wave_equals_serial(qdriver, seed, L1, L2):
    """The threaded MEA (bands of 64 rows pipelined over threads, for large
    profiles) against the serial recurrence (ProbabilisticModel::
    computeAlignment): same path and score."""
    out = subprocess.run([qdriver, 'mea', str(seed), str(L1), str(L2)], capture_output=True, text=True, check=True)
    assert out.stdout.strip() == 'same'
