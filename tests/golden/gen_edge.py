"""Golden outputs of both reference CLIs on small edge-case families
(tests/golden/edge): two sequences, single-residue sequences, identical
sequences, lower case and X/B/Z letters.  Made with the reference CLIs built
from source (oracle/_ref: `make -C oracle ref qp`); c_p_np_aln single-thread.
Usage: python tests/golden/gen_edge.py
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, 'edge')
REFCLI = os.path.join(ROOT, 'oracle', '_ref', 'c_p_np_aln')
QPCLI = os.path.join(ROOT, 'oracle', '_ref', 'quickprobs')

FAMILIES = {
    'two': '>a\nMKV\n>b\nMKVL\n',
    'short': '>s1\nM\n>s2\nMK\n>s3\nW\n>s4\nMKVLAG\n',
    'dup': '>d1\nMKVLAAGIVGLLLAQW\n>d2\nMKVLAAGIVGLLLAQW\n>d3\nMKVLAAGIVGLLLAQW\n>d4\nMKVLGAGIVLLAQ\n',
    'mixed': '>low case\nmkvlaagivg\nlllaqw\n>x2  \nMKVXLBAZGHWKQ\n>x3\nmkvlgagivllaqwxxbz\n',
    'crlf': '>c1 header\r\nMKVLAAGIVG\r\nLLLAQW\r\n>c2\r\nMKVLGAGIVLLAQ\r\n>c3\r\nMKKLAAGIVGLL\r\n',
}


def main():
    os.makedirs(OUT, exist_ok=True)
    for name, text in FAMILIES.items():
        fa = os.path.join(OUT, name + '.fa')
        with open(fa, 'w', newline='') as fh:
            fh.write(text)
        for tag, cmd in (('G', ['taskset', '-c', '0', REFCLI, '-G', fa]),
                         ('p_0', ['taskset', '-c', '0', REFCLI, '-p', '0', fa]),
                         ('qp', [QPCLI, fa])):
            r = subprocess.run(cmd, capture_output=True)
            assert r.returncode == 0, (name, tag, r.stderr)
            with open(os.path.join(OUT, f'{name}.{tag}.out'), 'wb') as fh:
                fh.write(r.stdout)
            print(name, tag, len(r.stdout))


if __name__ == '__main__':
    main()
