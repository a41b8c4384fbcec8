"""Golden outputs of both reference CLIs on real benchmark families.

Families are taken from the reference's own benchmark inputs
(/root/reference/TEST/{bali3,ox,oxx,sabre}/in; data files, copied verbatim
into tests/golden/real/), a deterministic sample of small ones (every k-th
file by name with at most 4e6 pair-cells, so the single-thread reference run
stays short).  For each family:
  c_p_np_aln -G and -p 0   oracle/_ref/c_p_np_aln (the reference C_P_NP_Aln
                           sources, `make -C oracle ref`), single thread
                           (taskset -c 0: the reference's races)
  quickprobs               oracle/_ref/quickprobs (the reference QuickProbs
                           sources, `make -C oracle qp`); exit status kept,
                           QuickProbs rejects '-' in its input.
plus 8 larger oxx families (60-420 sequences) for quickprobs only.
Usage: python tests/golden/gen_real.py
"""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
TEST = '/root/reference/TEST'
OUT = os.path.join(HERE, 'real')
REFCLI = os.path.join(ROOT, 'oracle', '_ref', 'c_p_np_aln')
QPCLI = os.path.join(ROOT, 'oracle', '_ref', 'quickprobs')


def seqs_of(path):
    txt = open(path).read()
    out = []
    for rec in txt.split('>')[1:]:
        body = rec.split('\n', 1)[1] if '\n' in rec else ''
        out.append(''.join(c for c in body if c.isalpha()))
    return out


def pair_cells(seqs):
    L = [len(s) for s in seqs]
    return sum((L[a] + 1) * (L[b] + 1) for a in range(len(L)) for b in range(a + 1, len(L)))


def main():
    os.makedirs(OUT, exist_ok=True)
    man = []
    for d in ('bali3', 'ox', 'oxx', 'sabre'):
        files = sorted(os.listdir(os.path.join(TEST, d, 'in')))
        picked = 0
        for k, f in enumerate(files):
            if picked >= 10:
                break
            src = os.path.join(TEST, d, 'in', f)
            s = seqs_of(src)
            if k % 7 != 0 or len(s) < 2 or pair_cells(s) > 4e6:
                continue
            picked += 1
            name = f'{d}_{f}'
            dst = os.path.join(OUT, name + '.fa')
            with open(src, 'rb') as fi, open(dst, 'wb') as fo:
                fo.write(fi.read())
            ent = {'family': name, 'n': len(s), 'pair_cells': pair_cells(s)}
            for tag, cmd in (('G', ['taskset', '-c', '0', REFCLI, '-G', dst]),
                             ('p_0', ['taskset', '-c', '0', REFCLI, '-p', '0', dst]),
                             ('qp', [QPCLI, '-t', '4', dst])):
                r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
                with open(os.path.join(OUT, f'{name}.{tag}.out'), 'w') as fh:
                    fh.write(r.stdout)
                ent[tag] = {'rc': r.returncode, 'stderr': r.stderr[-200:]}
            man.append(ent)
            print(name, ent['n'], ent['pair_cells'], {t: ent[t]['rc'] for t in ('G', 'p_0', 'qp')}, flush=True)
    # larger families for the quickprobs drop-in only (its output does not
    # depend on the thread count): > 50 sequences (1 consistency round), > 200
    # (selectivity rejects z, 200 refinement passes)
    files = sorted(os.listdir(os.path.join(TEST, 'oxx', 'in')))
    picked = 0
    for k, f in enumerate(files):
        src = os.path.join(TEST, 'oxx', 'in', f)
        s = seqs_of(src)
        if picked >= 8 or k % 5 != 0 or not (60 <= len(s) <= 420) or pair_cells(s) > 2e9:
            continue
        picked += 1
        name = f'oxxL_{f}'
        dst = os.path.join(OUT, name + '.fa')
        with open(src, 'rb') as fi, open(dst, 'wb') as fo:
            fo.write(fi.read())
        r = subprocess.run([QPCLI, '-t', '8', dst], capture_output=True, text=True, timeout=1800)
        with open(os.path.join(OUT, f'{name}.qp.out'), 'w') as fh:
            fh.write(r.stdout)
        ent = {'family': name, 'n': len(s), 'pair_cells': pair_cells(s), 'qp': {'rc': r.returncode,
                                                                                'stderr': r.stderr[-200:]}}
        man.append(ent)
        print(name, ent['n'], ent['pair_cells'], r.returncode, flush=True)
    with open(os.path.join(OUT, 'manifest.json'), 'w') as fh:
        json.dump(man, fh, indent=1)


if __name__ == '__main__':
    main()
