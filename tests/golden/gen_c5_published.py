"""The published MLProbs outputs (the reference's output4evaluation/<bench>/
<family>) of the C5 bench sample -- every 15th TEST/ox + TEST/sabre family of
tests/golden/sweep.json.xz, bench.py's c5 leg -- as data for the bench's
SP / TC readouts on the GPU box (the reference tree is not there).

    python tests/golden/gen_c5_published.py [/root/reference]
"""
import json
import lzma
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REF = sys.argv[1] if len(sys.argv) > 1 else '/root/reference'


def c5_names(fams):
    return [k for k in sorted(fams) if k.split('/')[0] in ('ox', 'sabre') and 'p_0' in fams[k]][::15]


def main():
    with lzma.open(os.path.join(HERE, 'sweep.json.xz'), 'rt') as fh:
        fams = json.load(fh)
    out = {}
    for name in c5_names(fams):
        bench, fam = name.split('/')
        with open(os.path.join(REF, 'output4evaluation', bench, fam), encoding='latin-1') as fh:
            out[name] = fh.read()
    with lzma.open(os.path.join(HERE, 'c5_published.json.xz'), 'wt') as fh:
        json.dump(out, fh)
    print(len(out), 'families')


if __name__ == '__main__':
    main()
