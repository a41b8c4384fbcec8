"""Parity sweep on the GPU box: both drop-in CLIs over every family in
tests/golden/sweep.json.xz (the reference's own benchmark families with the
outputs of the reference CLIs built from source, tools/gen_sweep.py),
compared byte for byte.  Runs `workers` CLI processes at a time (8 GB batch
scratch each) and writes a summary and any mismatches to OUT.  TAGS (comma
list of G, p_0, qp; default all) selects the runs: the c_p_np_aln runs of
the sweep (G, p_0; at most 2e6 pair-cells) all take the drop-in's host path
(mlp_ctx_create_host), so `G,p_0` needs no GPU.
With MAX_CELLS only families of at most that many pair-cells run (the
drop-ins' host path: `qp 4e6` runs without a GPU).
    python tools/parity_sweep.py OUT [workers] [TAGS] [MAX_CELLS]
"""
import json
import lzma
import os
import subprocess
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CP = os.path.join(ROOT, 'mlprobs_amd', 'cli', 'c_p_np_aln')
QP = os.path.join(ROOT, 'mlprobs_amd', 'cli', 'quickprobs')


def pair_cells(fa_text):
    """(L_a + 1)(L_b + 1) summed over pairs, residues as the CLIs count them."""
    lens, cur = [], None
    for line in fa_text.splitlines():
        if line.startswith('>'):
            if cur is not None:
                lens.append(cur)
            cur = 0
        elif cur is not None:
            cur += sum(ch.isalpha() for ch in line)
    if cur is not None:
        lens.append(cur)
    tot = sum(lens)
    return ((tot + len(lens)) ** 2 - sum((L + 1) ** 2 for L in lens)) / 2


def main():
    out = sys.argv[1]
    workers = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    tags = sys.argv[3].split(',') if len(sys.argv) > 3 else ['G', 'p_0', 'qp']
    max_cells = float(sys.argv[4]) if len(sys.argv) > 4 else float('inf')
    with lzma.open(os.path.join(ROOT, 'tests', 'golden', 'sweep.json.xz'), 'rt') as fh:
        fams = json.load(fh)
    env = dict(os.environ, MLP_SCRATCH_GB='8', MLP_HOST_THREADS='2')
    td = tempfile.mkdtemp()
    jobs = []
    for name, e in sorted(fams.items()):
        if pair_cells(e['fa']) > max_cells:
            continue
        fa = os.path.join(td, name.replace('/', '_') + '.fa')
        with open(fa, 'wb') as fh:
            fh.write(e['fa'].encode('latin-1'))
        for tag, cmd in (('G', [CP, '-G', fa]), ('p_0', [CP, '-p', '0', fa]), ('qp', [QP, fa])):
            if tag in e and tag in tags:
                jobs.append((name, tag, cmd, e[tag]))

    def run(job):
        name, tag, cmd, (rc, ref) = job
        r = subprocess.run(cmd, capture_output=True, timeout=600, env=env)
        got = r.stdout.decode('latin-1')
        ok = (r.returncode == 0) == (rc == 0) and (rc != 0 or got == ref)
        return name, tag, ok, r.returncode, rc, rc != 0 and r.returncode != 0

    t0 = time.time()
    res = []
    with ThreadPoolExecutor(workers) as ex:
        for i, x in enumerate(ex.map(run, jobs)):
            res.append(x)
            if i % 200 == 0:
                print(f'{i}/{len(jobs)} {time.time() - t0:.0f} s', flush=True)
    bad = [x for x in res if not x[2]]
    by = {}
    for name, tag, ok, _, _, both_fail in res:
        s = by.setdefault(tag, [0, 0, 0])
        s[0] += ok and not both_fail
        s[1] += 1
        s[2] += both_fail
    with open(out, 'w') as fh:
        fh.write(f'families {len(fams)}, runs {len(res)}, {time.time() - t0:.0f} s\n')
        for tag, (ok, n, nf) in sorted(by.items()):
            fh.write(f'{tag}: {ok}/{n} byte-identical, {nf} failing in both (reference and drop-in exit != 0)\n')
        for name, tag, ok, rc, rrc, _ in bad:
            fh.write(f'MISMATCH {name} {tag} rc {rc} (reference {rrc})\n')
    print(open(out).read())


if __name__ == '__main__':
    main()
