"""Golden outputs of the reference CLI's non-progressive strategy (-p 1,
MSA::npdoAlign, CPNP/MSA.cpp:1084-1140) and of its pair loop.

* tests/golden/np/<family>.p_1_ir_0.out: oracle/_ref/c_p_np_aln -p 1 -ir 0
  (alignment graph only: deterministic), single thread (taskset -c 0);
* tests/golden/np/<family>.p_1.out: oracle/_ref/c_p_np_aln_ft -p 1 (the
  reference CLI with time() fixed at REF_FIXED_TIME = 1700000000 by
  oracle/fixtime.c, so its srand(time(0)) refinement is reproducible; the
  drop-in takes the same clock from MLP_SRAND_TIME);
* tests/golden/np_pairs_<family>.npz: ref_probe npdo (the reference's own
  ArrangePosteriorProbs over every pair at the family's pid / delta):
  distances score / #B and the CSR.
Families: the three CLI goldens and the real benchmark families of
tests/golden/real (those whose -p 1 reference run takes < 60 s).
Usage: python tests/golden/gen_np.py
"""
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
REFCLI = os.path.join(ROOT, 'oracle', '_ref', 'c_p_np_aln')
REFFT = os.path.join(ROOT, 'oracle', '_ref', 'c_p_np_aln_ft')
PROBE = os.path.join(ROOT, 'oracle', '_ref', 'ref_probe')
OUT = os.path.join(HERE, 'np')
TIME = '1700000000'
TIMEOUT = float(os.environ.get('NP_TIMEOUT', '60'))  # families whose reference run is slower are skipped


def run(cmd, env=None, timeout=120):
    return subprocess.run(['taskset', '-c', '0'] + cmd, capture_output=True, timeout=timeout,
                          env=dict(os.environ, **(env or {})))


def main():
    import bench  # read_pair_dump
    import orc
    from mlprobs_amd import synth
    os.makedirs(OUT, exist_ok=True)
    fams = [(n, os.path.join(HERE, 'cli', n + '.fa')) for n in ('div12', 'sim8', 'bb11028')]
    real = sorted(f[:-3] for f in os.listdir(os.path.join(HERE, 'real')) if f.endswith('.fa'))
    fams += [(n, os.path.join(HERE, 'real', n + '.fa')) for n in real]
    edge = sorted(f[:-3] for f in os.listdir(os.path.join(HERE, 'edge')) if f.endswith('.fa'))
    fams += [(n, os.path.join(HERE, 'edge', n + '.fa')) for n in edge]
    only = sys.argv[1:]  # optional: family names to (re)generate
    fams = [f for f in fams if not only or f[0] in only]
    man = []
    for name, fa in fams:
        ent = {'family': name}
        try:
            r0 = run([REFCLI, '-p', '1', '-ir', '0', fa], timeout=TIMEOUT)
            r1 = run([REFFT, '-p', '1', fa], env={'REF_FIXED_TIME': TIME}, timeout=TIMEOUT)
        except subprocess.TimeoutExpired:
            print(name, 'skipped (slow)', flush=True)
            continue
        for tag, r in (('p_1_ir_0', r0), ('p_1', r1)):
            with open(os.path.join(OUT, f'{name}.{tag}.out'), 'wb') as fh:
                fh.write(r.stdout)
            ent[tag] = r.returncode
        man.append(ent)
        print(name, ent, flush=True)
    # pair-loop fixtures (oracle pin): pid / delta from the family test
    for name in ('div12', 'sim8', 'bb11028'):
        if only and name not in only:
            continue
        fa = os.path.join(HERE, 'cli', name + '.fa')
        seqs = [s for _, s in synth.read_fasta(fa)]
        vm, _, delta = orc.model_adjustment(orc.model(0.132548), seqs)
        pid = vm % 10
        dump = '/tmp/np_dump.bin'
        subprocess.check_call([PROBE, 'npdo', fa, str(pid), repr(delta), dump])
        d = bench.read_pair_dump(dump)
        np.savez_compressed(os.path.join(HERE, f'np_pairs_{name}.npz'), pid=pid, delta=np.float32(delta),
                            ab=np.array(d['ab'], np.int32), L1=d['L1'], dist=d['dist'], rp=d['rp'],
                            eoff=d['eoff'], cols=d['cols'], vals=d['vals'])
        man.append({'pairs': name, 'pid': int(pid), 'delta': float(delta), 'npairs': len(d['ab'])})
    path = os.path.join(OUT, 'manifest.json')
    if only and os.path.exists(path):  # merge into the existing manifest
        with open(path) as fh:
            old = json.load(fh)['entries']
        keep = [e for e in old if e.get('family') not in only and e.get('pairs') not in only]
        man = keep + man
    with open(path, 'w') as fh:
        json.dump({'fixed_time': int(TIME), 'entries': man}, fh, indent=1)


if __name__ == '__main__':
    main()
