"""Seeded synthetic protein families.

Root of length L drawn i.i.d. from the ProbCons background distribution
(CPNP/Defaults.h emitSingleDefault); each of N descendants walks the root:
deletion w.p. `indel/2`, otherwise substitution w.p. `s` (resampled from the
background), then an insertion of one background residue w.p. `indel/2`.
Headers are ``s%04d``.  s=0.7 gives identity ~0.15 (pid 0, every model runs).
"""
import numpy as np

ALPHABET = 'ARNDCQEGHILKMFPSTWYV'
# ProbCons background frequencies, alphabet order (CPNP/Defaults.h:30-34).
BACKGROUND = np.array([
    0.07831005, 0.05246024, 0.04433257, 0.05130349, 0.02189704, 0.03585766,
    0.05615771, 0.07783433, 0.02601093, 0.06511648, 0.09716489, 0.05877077,
    0.02438117, 0.04463228, 0.03940142, 0.05849916, 0.05115306, 0.01203523,
    0.03124726, 0.07343426])
BACKGROUND = BACKGROUND / BACKGROUND.sum()
_LETTERS = np.frombuffer(ALPHABET.encode(), np.uint8)


def family(n, length, s, seed, indel=0.05):
    """Return a list of (header, sequence) tuples."""
    rng = np.random.default_rng(seed)
    root = rng.choice(20, size=length, p=BACKGROUND)
    out = []
    for d in range(n):
        keep = rng.random(length) >= indel / 2
        sub = rng.random(length) < s
        res = np.where(sub, rng.choice(20, size=length, p=BACKGROUND), root)
        ins = rng.random(length) < indel / 2
        insres = rng.choice(20, size=length, p=BACKGROUND)
        seq = []
        for k in range(length):
            if keep[k]:
                seq.append(res[k])
            if ins[k]:
                seq.append(insres[k])
        if not seq:
            seq = [root[0]]
        out.append(('s%04d' % d, _LETTERS[np.array(seq)].tobytes().decode()))
    return out


def write_fasta(path, fam, width=60):
    with open(path, 'w') as fh:
        for h, s in fam:
            fh.write('>' + h + '\n')
            for i in range(0, len(s), width):
                fh.write(s[i:i + width] + '\n')


def read_fasta(path):
    """Minimal MFA reader mirroring CPNP/Sequence.h:54-125 for clean input."""
    fam, h, buf = [], None, []
    with open(path) as fh:
        for line in fh:
            line = line.rstrip('\n')
            if line.startswith('>'):
                if h is not None:
                    fam.append((h, ''.join(buf)))
                h, buf = line[1:].strip(), []
            else:
                buf.append(''.join(ch for ch in line if not ch.isspace()).replace('.', '-')
                           .replace('-', '').upper())
    if h is not None:
        fam.append((h, ''.join(buf)))
    return fam
