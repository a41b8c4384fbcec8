"""Reference outputs for a parity sweep over the reference's own benchmark
families (TEST/{bali3,ox,oxx,sabre}/in), for tools/parity_sweep.py.

Runs the reference CLIs built from source (oracle/_ref) on every family up to
a size bound: quickprobs on families with <= 4e7 pair-cells (its output does
not depend on the thread count; 1 thread per process here), c_p_np_aln -G and
-p 0 single-threaded (taskset) on families with <= 2e6 pair-cells.  Inputs and
outputs go to tests/golden/sweep.json.xz (the inputs are the reference's data
files, verbatim).  Usage: python tools/gen_sweep.py [workers]
"""
import json
import lzma
import os
import subprocess
import sys
from multiprocessing import Pool

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TEST = '/root/reference/TEST'
REFCLI = os.path.join(ROOT, 'oracle', '_ref', 'c_p_np_aln')
QPCLI = os.path.join(ROOT, 'oracle', '_ref', 'quickprobs')
OUT = os.path.join(ROOT, 'tests', 'golden', 'sweep.json.xz')


def seqs_of(text):
    out = []
    for rec in text.split('>')[1:]:
        body = rec.split('\n', 1)[1] if '\n' in rec else ''
        out.append(''.join(c for c in body if c.isalpha()))
    return out


def cells(s):
    L = [len(x) for x in s]
    return sum((L[a] + 1) * (L[b] + 1) for a in range(len(L)) for b in range(a + 1, len(L)))


def work(args):
    k, name, path = args
    text = open(path, 'rb').read().decode('latin-1')
    s = seqs_of(text)
    c = cells(s)
    ent = {'fa': text, 'n': len(s), 'cells': c}
    cpu = str(k % 8)
    if len(s) >= 2 and c <= 4e7:
        r = subprocess.run([QPCLI, '-t', '1', path], capture_output=True, timeout=3600)
        ent['qp'] = [r.returncode, r.stdout.decode('latin-1')]
    if len(s) >= 2 and c <= 2e6:
        for tag, extra in (('G', ['-G']), ('p_0', ['-p', '0'])):
            r = subprocess.run(['taskset', '-c', cpu, REFCLI] + extra + [path], capture_output=True, timeout=3600)
            ent[tag] = [r.returncode, r.stdout.decode('latin-1')]
    return name, ent


def main():
    workers = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    jobs = []
    for d in ('bali3', 'ox', 'oxx', 'sabre'):
        for f in sorted(os.listdir(os.path.join(TEST, d, 'in'))):
            jobs.append((len(jobs), f'{d}/{f}', os.path.join(TEST, d, 'in', f)))
    res = {}
    with Pool(workers) as pool:
        for i, (name, ent) in enumerate(pool.imap_unordered(work, jobs, chunksize=4)):
            res[name] = ent
            if i % 100 == 0:
                print(i, name, flush=True)
    with lzma.open(OUT, 'wt') as fh:
        json.dump(res, fh)
    print('families', len(res), 'qp', sum('qp' in e for e in res.values()),
          'cpnp', sum('p_0' in e for e in res.values()))


if __name__ == '__main__':
    main()
