"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself.

Runs oracle/_ref/ref_probe (the reference C_P_NP_Aln objects compiled in place
from /root/reference by `make -C oracle ref`) and oracle/_ref/c_p_np_aln on
seeded synthetic inputs (mlprobs_amd/synth.py) and on TEST/bali3 family
BB11028, and stores inputs + reference outputs as compressed .npz / text.
Only runnable in the build container (needs /root/reference); the fixtures
it writes are committed and are all the GPU box ever sees.

    python tests/golden/gen_golden.py
"""
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tools'))
import refdump  # noqa: E402
from mlprobs_amd import synth  # noqa: E402

PROBE = os.path.join(ROOT, 'oracle', '_ref', 'ref_probe')
REFCLI = os.path.join(ROOT, 'oracle', '_ref', 'c_p_np_aln')
BALI = '/root/reference/TEST/bali3/in/BB11028'


def probe(args, td):
    out = os.path.join(td, 'o.bin')
    subprocess.check_call([PROBE] + [str(a) for a in args], env=dict(os.environ, REF_PROBE_OUT=out))
    return refdump.read(out)


def to_rowptr(rowsize):
    rs = np.asarray(rowsize, np.int64)
    rp = np.zeros(len(rs) + 1, np.int32)
    rp[2:] = np.cumsum(rs[1:])
    return rp


def gen_params(td):
    res = {}
    for tag, delta in (('default', None), ('d170705', 0.170705)):
        d = probe(['params'] + ([delta] if delta is not None else []), td)
        for k in ('initialDistribution', 'transProb', 'matchProb', 'insProb',
                  'local_transProb', 'random_transProb'):
            res[f'{tag}.{k}'] = d[k]
        res['sub_matrix'] = d['sub_matrix']
        res['subst_index'] = d['subst_index']
    np.savez_compressed(os.path.join(HERE, 'params.npz'), **res)


PAIR_CASES = []


def _pair_cases():
    cases = [
        ('tiny_aa', 'A', 'A', -1),
        ('tiny_w4', 'W', 'ACDE', -1),
        ('tiny_6_1', 'ACDEFG', 'K', 0.170705),
        ('xbz', 'MKVXLBAZGHW', 'MKVLLDAEGHWQ', -1),
    ]
    f = synth.family(4, 30, 0.7, seed=1)
    cases.append(('div30', f[0][1], f[1][1], 0.132548))
    f = synth.family(4, 60, 0.5, seed=2)
    cases.append(('mid60', f[1][1], f[3][1], 0.100675))
    f = synth.family(3, 90, 0.2, seed=3)
    cases.append(('sim90', f[0][1], f[2][1], -1))
    g = synth.family(2, 20, 0.3, seed=4)
    h = synth.family(2, 75, 0.3, seed=5)
    cases.append(('ragged', g[0][1], h[1][1], 0.168284))
    cases.append(('ragged_t', h[1][1], g[0][1], 0.168284))
    return cases


def gen_pairs(td):
    manifest = []
    for name, s1, s2, delta in _pair_cases():
        fa = os.path.join(td, 'p.fa')
        synth.write_fasta(fa, [('a', s1), ('b', s2)])
        d0 = delta
        if delta < 0:
            d0 = float(np.float32(0.700645))  # initDistrib2Default[2] (CPNP/Defaults.h:23)
        d = probe(['pair', fa, 0, 1, repr(d0)], td)
        out = {'s1': np.frombuffer(s1.encode(), np.uint8), 's2': np.frombuffer(s2.encode(), np.uint8),
               'delta': np.float32(d0)}
        for k, v in d.items():
            if k.endswith('.rowsize'):
                out[k[:-8] + '.rowptr'] = to_rowptr(v)
            else:
                out[k] = v
        np.savez_compressed(os.path.join(HERE, f'pair_{name}.npz'), **out)
        manifest.append({'name': name, 'L1': len(s1), 'L2': len(s2), 'delta': d0})
    return manifest


def gen_family(td, name, fam, reps, pid_override=-1):
    fa = os.path.join(td, 'f.fa')
    synth.write_fasta(fa, fam)
    d = probe(['family', fa, reps, pid_override, 1], td)
    n = int(d['N'][0])
    P = n * (n - 1) // 2
    out = {'seqs': np.array([s for _, s in fam]), 'lens': d['lens'], 'variance_mean': d['variance_mean'],
           'delta': d['delta'], 'pid': d['pid'], 'distances': d['distances'].reshape(n, n),
           'mea': d['mea'].reshape(n, n)}
    for it in range(reps + 1):
        rps, cols, vals = [], [], []
        for p in range(P):
            rps.append(to_rowptr(d[f'it{it}.p{p}.rowsize']))
            cols.append(d[f'it{it}.p{p}.cols'])
            vals.append(d[f'it{it}.p{p}.vals'])
        out[f'it{it}.rowptr'] = np.concatenate(rps)
        out[f'it{it}.cols'] = np.concatenate(cols)
        out[f'it{it}.vals'] = np.concatenate(vals)
    out['reps'] = np.int32(reps)
    np.savez_compressed(os.path.join(HERE, f'family_{name}.npz'), **out)
    return {'name': name, 'N': n, 'reps': reps, 'pid': int(d['pid'][0]),
            'variance_mean': int(d['variance_mean'][0]), 'delta': float(d['delta'][0])}


def gen_cli(td):
    """Reference CLI outputs, single-threaded (taskset -c 0: the reference sets
    its thread count from omp_get_num_procs(), CPNP/MSA.cpp:147-151)."""
    outdir = os.path.join(HERE, 'cli')
    os.makedirs(outdir, exist_ok=True)
    cases = {'bb11028.fa': None,
             'div12.fa': synth.family(12, 60, 0.7, seed=21),
             'sim8.fa': synth.family(8, 80, 0.2, seed=22)}
    man = []
    for fname, fam in cases.items():
        src = os.path.join(outdir, fname)
        if fam is None:
            shutil.copyfile(BALI, src)
        else:
            synth.write_fasta(src, fam)
        for args in (['-G'], ['-p', '0'], ['-p', '0', '-c', '0', '-ir', '0']):
            r = subprocess.run(['taskset', '-c', '0', REFCLI] + args + [src], capture_output=True, text=True)
            tag = fname[:-3] + '_' + '_'.join(a.strip('-') for a in args)
            with open(os.path.join(outdir, tag + '.out'), 'w') as fh:
                fh.write(r.stdout)
            man.append({'input': fname, 'args': args, 'out': tag + '.out', 'rc': r.returncode,
                        'stderr': r.stderr})
    return man


QPPROBE = os.path.join(ROOT, 'oracle', '_ref', 'qp_probe')
QPCLI = os.path.join(ROOT, 'oracle', '_ref', 'quickprobs')


def gen_qp_cli():
    """Reference QuickProbs CLI outputs (oracle/_ref/quickprobs: QP/Console/
    main.cpp built from the reference sources by `make -C oracle qp`; its
    output does not depend on the thread count)."""
    outdir = os.path.join(HERE, 'cli')
    extra = {'qp_div60.fa': synth.family(60, 50, 0.6, seed=41),     # > 50 sequences: 1 consistency round
             'qp_big210.fa': synth.family(210, 30, 0.5, seed=42)}   # > 200: selectivity rejects z, 200 passes
    for fname, fam in extra.items():
        synth.write_fasta(os.path.join(outdir, fname), fam)
    cases = [('bb11028.fa', []), ('bb11028.fa', ['-c', '0']), ('bb11028.fa', ['-c', '1', '-r', '5']),
             ('div12.fa', []), ('div12.fa', ['-c', '0']), ('sim8.fa', []), ('sim8.fa', ['-c', '3', '-r', '50']),
             ('qp_div60.fa', []), ('qp_big210.fa', [])]
    man = []
    for fname, args in cases:
        r = subprocess.run([QPCLI] + args + [os.path.join(outdir, fname)], capture_output=True, text=True)
        tag = 'qp_' + fname[:-3].replace('qp_', '') + ''.join('_' + a.strip('-') for a in args)
        with open(os.path.join(outdir, tag + '.out'), 'w') as fh:
            fh.write(r.stdout)
        man.append({'input': fname, 'args': args, 'out': tag + '.out', 'rc': r.returncode, 'stderr': r.stderr})
    return man


def gen_qp(td):
    """QuickProbs posterior-stage vectors (oracle/_ref/qp_probe, the reference
    QuickProbs sources compiled in place by `make -C oracle qp`)."""
    cases = [
        ('tiny', 'A', 'W'),
        ('xbz', 'MKVXLBAZGHWJ', 'MKVLLDAEGHWQOU'),
        ('short', 'MKVLAAGIVGLLLAQ', 'MKVLGAGIVLLAQW'),
    ]
    f = synth.family(4, 60, 0.7, seed=21)
    cases.append(('div60', f[0][1], f[2][1]))
    f = synth.family(4, 120, 0.45, seed=22)
    cases.append(('mid120', f[1][1], f[3][1]))
    f = synth.family(3, 200, 0.15, seed=23)
    cases.append(('sim200', f[0][1], f[1][1]))
    g = synth.family(2, 25, 0.4, seed=24)
    h = synth.family(2, 300, 0.4, seed=25)
    cases.append(('ragged', g[0][1], h[1][1]))
    cases.append(('ragged_t', h[1][1], g[0][1]))
    manifest = []
    for name, s1, s2 in cases:
        out = os.path.join(td, 'q.bin')
        subprocess.check_call([QPPROBE, 'pair', s1, s2], env=dict(os.environ, REF_PROBE_OUT=out))
        d = refdump.read(out)
        d['s1'] = np.frombuffer(s1.encode(), np.uint8)
        d['s2'] = np.frombuffer(s2.encode(), np.uint8)
        np.savez_compressed(os.path.join(HERE, f'qp_pair_{name}.npz'), **d)
        manifest.append({'name': name, 'L1': len(s1), 'L2': len(s2)})
    return manifest


def gen_qp_relax(td):
    """QuickProbs' posterior stage + consistency rounds on small families
    (qp_probe relax: PosteriorStage, then ConsistencyStage::doRelaxation with
    the default configuration, the last round unfiltered)."""
    rng = np.random.default_rng(31)
    fams = [
        ('mid6', synth.family(6, 60, 0.5, seed=31), 2, None),
        ('div8', synth.family(8, 80, 0.7, seed=32), 2, None),
        ('ragged7', [(h, s[: 12 + 11 * i]) for i, (h, s) in enumerate(synth.family(7, 90, 0.4, seed=33))], 1, None),
        # the selectivity filter rejecting z: threshold = the median posterior
        # distance (ConsistencyStage.cpp:171-205)
        ('sel9', synth.family(9, 70, 0.5, seed=34), 2, 'median'),
    ]
    manifest = []
    for name, fam, iters, sel in fams:
        seqs = [s for _, s in fam]
        w = rng.uniform(0.5, 20.0, len(seqs)).astype(np.float32)
        path = os.path.join(td, 'r.txt')
        with open(path, 'w') as fh:
            for wt, sq in zip(w, seqs):
                fh.write(f'{float(wt)!r} {sq}\n')
        out = os.path.join(td, 'r.bin')
        args = [QPPROBE, 'relax', path, str(iters)]
        if sel == 'median':
            subprocess.check_call(args, env=dict(os.environ, REF_PROBE_OUT=out))
            args.append(repr(float(np.median(refdump.read(out)['dist']))))
        subprocess.check_call(args, env=dict(os.environ, REF_PROBE_OUT=out))
        d = refdump.read(out)
        d['seqs'] = np.array(seqs)
        d['weights'] = w
        d['iters'] = np.int32(iters)
        np.savez_compressed(os.path.join(HERE, f'qp_family_{name}.npz'), **d)
        manifest.append({'name': name, 'n': len(seqs), 'iters': iters,
                         'selectivity': float(d['selectivity'][0])})
    return manifest


def main():
    if '--qpcli' in sys.argv:  # QuickProbs CLI outputs only (merged into the manifest)
        path = os.path.join(HERE, 'manifest.json')
        with open(path) as fh:
            man = json.load(fh)
        man['qp_cli'] = gen_qp_cli()
        with open(path, 'w') as fh:
            json.dump(man, fh, indent=1)
        return
    if '--qp' in sys.argv:  # QuickProbs vectors only (merged into the manifest)
        with tempfile.TemporaryDirectory() as td:
            qp = gen_qp(td)
            qpf = gen_qp_relax(td)
        path = os.path.join(HERE, 'manifest.json')
        with open(path) as fh:
            man = json.load(fh)
        man['qp_pairs'] = qp
        man['qp_families'] = qpf
        man['qp_reference'] = '/root/reference realign/QuickProbs/src, oracle/Makefile `make qp`'
        with open(path, 'w') as fh:
            json.dump(man, fh, indent=1)
        return
    with tempfile.TemporaryDirectory() as td:
        gen_params(td)
        pairs = gen_pairs(td)
        fams = [
            gen_family(td, 'div8', synth.family(8, 40, 0.7, seed=11), 3),
            gen_family(td, 'div8_pid2', synth.family(8, 40, 0.7, seed=11), 2, 2),
            gen_family(td, 'div8_pid3', synth.family(8, 40, 0.7, seed=11), 2, 3),
            gen_family(td, 'mid6', synth.family(6, 50, 0.45, seed=12), 2),
            gen_family(td, 'sim6', synth.family(6, 60, 0.2, seed=13), 2),
            gen_family(td, 'ragged7', [(h, s[: 10 + 9 * i]) for i, (h, s) in
                                      enumerate(synth.family(7, 70, 0.6, seed=14))], 2),
        ]
        bali = synth.read_fasta(BALI)
        fams.append(gen_family(td, 'bb11028', bali, 2))
        cli = gen_cli(td)
        qp = gen_qp(td)
        qpf = gen_qp_relax(td)
    with open(os.path.join(HERE, 'manifest.json'), 'w') as fh:
        json.dump({'generator': 'tests/golden/gen_golden.py',
                   'reference': '/root/reference (kuangmeng/MLProbs v1), baseMSA/C_P_NP_Aln',
                   'build': 'oracle/Makefile `make ref` (CPNP/Makefile flags)',
                   'pairs': pairs, 'families': fams, 'cli': cli, 'qp_pairs': qp, 'qp_families': qpf,
                   'qp_reference': '/root/reference realign/QuickProbs/src, oracle/Makefile `make qp`'}, fh, indent=1)


if __name__ == '__main__':
    main()
