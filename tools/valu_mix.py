"""Mix-weighted VALU issue peak per bench kernel group: compiles
the kernels to gfx950 assembly, classes every VALU instruction of each kernel
full or half rate (tools/isa_mix.py, rates measured by tools/probe/valu_rate),
weights the kernels of a group by their measured VALU instruction counts
(SQ_INSTS_VALU of a PMC pass, tools/pmc_summary.py kernels.json) and writes
'valu_mix_peak' (wave-instr/s) and 'valu_half_frac' into the groups of the
traffic JSON that bench.py reads.

    python tools/valu_mix.py profiles/r05_pmc_kernels.json profiles/pmc_traffic.json
"""
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
sys.path.insert(0, os.path.join(ROOT, 'tools'))
import isa_mix  # noqa: E402

PEAK = 1.2288e12


def mangle(short):
    """k_forward<3> -> _ZN3mlp9k_forwardILi3E..., k_merge<7, 0, false> -> ..ILi7ELi0ELb0E.."""
    m = re.match(r'(k_\w+)(?:<(.*)>)?', short)
    base, args = m.group(1), m.group(2)
    s = f'_ZN3mlp{len(base)}{base}'
    if args:
        s += 'I'
        for a in (x.strip() for x in args.split(',')):
            s += {'false': 'Lb0E', 'true': 'Lb1E'}.get(a, f'Li{a}E')
        s += 'E'
    return s


def main():
    kern = json.load(open(sys.argv[1]))
    traffic_path = sys.argv[2]
    traffic = json.load(open(traffic_path))
    flags = ['--offload-arch=gfx950', '-O3', '-ffp-contract=off', '-fno-fast-math', '-fno-slp-vectorize', '-std=c++17',
             '--cuda-device-only', '-S', '-I', os.path.join(ROOT, 'include')]
    text = {}
    with tempfile.TemporaryDirectory() as td:
        for src in ('posterior.hip', 'totals.hip', 'relax.hip'):
            out = os.path.join(td, src + '.s')
            subprocess.run(['/opt/rocm/bin/hipcc'] + flags + [os.path.join(ROOT, 'mlprobs_amd', 'csrc', src), '-o', out],
                           check=True, capture_output=True)
            text[src] = open(out).read().splitlines()
    mix = {}
    for short in kern:
        if not short.startswith('k_'):
            continue
        pre = mangle(short)
        for src, lines in text.items():
            fn = next((l.split(':')[0] for l in lines if l.startswith(pre) and ':' in l and not l.startswith('\t')), None)
            if not fn:
                continue
            start = next(i for i, l in enumerate(lines) if l.startswith(fn + ':'))
            F = H = 0
            for l in lines[start + 1:]:
                l = l.strip()
                if l.startswith('.Lfunc_end'):
                    break
                c = isa_mix.classify(l) if l and not l.startswith(('.', ';')) else None
                F += c == 'full'
                H += c == 'half'
            if F + H:
                mix[short] = (F, H)
            break
    for g, e in traffic.items():
        if not isinstance(e, dict) or 'kernels' not in e:
            continue
        ks = [k for k in e['kernels'] if k in mix and kern[k].get('SQ_INSTS_VALU')]
        if not ks:
            continue
        insts = sum(kern[k]['SQ_INSTS_VALU'] for k in ks)
        # time-weighted: each kernel's instructions at its own mix's peak
        t = sum(kern[k]['SQ_INSTS_VALU'] * (mix[k][0] + 2 * mix[k][1]) / (mix[k][0] + mix[k][1]) / PEAK for k in ks)
        e['valu_mix_peak'] = insts / t
        e['valu_half_frac'] = {k: mix[k][1] / sum(mix[k]) for k in ks}
        print(g, f"{e['valu_mix_peak']:.3g}", e['valu_half_frac'])
    traffic['_valu_mix_note'] = ('valu_mix_peak: 1.23e12 wave-instr/s (2 cycles per wave64 instruction per SIMD) '
                                 'weighted by each kernel\'s full-rate / half-rate instruction mix in its compiled '
                                 'code (tools/valu_mix.py, rates from tools/probe/valu_rate)')
    with open(traffic_path, 'w') as fh:
        json.dump(traffic, fh, indent=1)


if __name__ == '__main__':
    main()
