"""VALU issue mix of a kernel's hot loop from a gfx950 .s file (hipcc
--save-temps / -S): each VALU instruction classed full rate (~2.4 SIMD cycles
per wave64 instruction at 8 waves per SIMD) or half rate (~4.4), by opcode and
operands, from tools/probe/valu_rate (profiles/r05e_valu_rate_opcodes.json):
full: v_add/sub/mul/fma_f32, v_add/sub_u32, v_and/or/xor, v_bitop3, v_mov_b32
with VGPR, literal or inline-constant operands; half: everything else (f32
max/min/med3, compares, v_cndmask, conversions, shifts, v_bcnt, 3-operand
integer ops, DPP, f64, packed f32) and any instruction with an SGPR source.
The mix-weighted issue peak is 1.23e12 x (F + H) / (F + 2H) wave-instr/s.

    python tools/isa_mix.py file.s FUNCTION_NAME [first_line last_line]
"""
import re
import sys

FULL = re.compile(r'^v_(add|sub|subrev|mul|fma)_f32|^v_(add|sub|subrev)_u32|^v_(and|or|xor)_b32|^v_bitop3_b32|^v_mov_b32_e32$|'
                  r'^v_mov_b32$|^v_add_co_u32|^v_mac_f32')


def classify(line):
    op = line.split()[0]
    if not op.startswith('v_') or op.startswith(('v_readlane', 'v_readfirstlane', 'v_writelane')):
        return None
    srcs = [x.strip() for x in line[len(op):].split(';')[0].split(',')[1:]]
    sgpr = any(re.match(r'^-?\|?(s\d+|s\[|vcc|exec|m0)', x) for x in srcs)
    dpp = 'dpp' in op or 'row_' in line or 'quad_perm' in line
    sdwa = 'sdwa' in op or 'dst_sel' in line
    if FULL.match(op) and not sgpr and not dpp and not sdwa:
        return 'full'
    return 'half'


def main():
    path, fn = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(fn + ':'))
    a, b = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (1, 10 ** 9)
    body = []
    for l in lines[start + a: start + b + 1]:
        if l.strip().startswith('.Lfunc_end'):
            break
        body.append(l.strip())
    F = H = 0
    for l in body:
        c = classify(l) if l else None
        if c == 'full':
            F += 1
        elif c == 'half':
            H += 1
    peak = 1.2288e12 * (F + H) / (F + 2 * H) if F + H else 0
    print(f'VALU {F + H}: full {F}, half {H} ({H / max(F + H, 1):.0%}); mix-weighted issue peak {peak:.3g} '
          f'wave-instr/s ({peak / 1.2288e12:.2f} of 1.23e12)')


if __name__ == '__main__':
    main()
