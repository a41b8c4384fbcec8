"""Exhaustive check of mlp_div3 (mlp_numerics.h): x / 3 as q = RN(x * RN(1/3)),
e = fma(-q, 3, x), fma(e, RN(1/3), q), against the IEEE quotient RN(x / 3),
emulated exactly on the CPU in float64: x - 3q is exact in float64 (26-bit
operands a few binades apart), e * r is exact (24 x 24 bits); q + e * r is
rounded once to float64 and then to float32, which differs from one rounding
only when the float64 value is exactly a float32 midpoint -- counted
separately (`ties`, none occur).

    python tools/check_div3.py [lo hi]      (float bit patterns; default [0, 3])
"""
import sys
import time

import numpy as np

R32 = np.float32(1.0) / np.float32(3.0)
R64 = np.float64(R32)


def check(lo, hi, step=1 << 24):
    bad = ties = 0
    for s in range(lo, hi, step):
        x = np.arange(s, min(s + step, hi), dtype=np.uint32).view(np.float32)
        bad_s, ties_s = check_values(x)
        bad += bad_s
        ties += ties_s
    return bad, ties


def check_values(x):
    x = np.asarray(x, np.float32)
    ref = x / np.float32(3.0)
    q = x * R32
    e = (x.astype(np.float64) - 3.0 * q.astype(np.float64)).astype(np.float32)
    s64 = q.astype(np.float64) + e.astype(np.float64) * R64
    q2 = s64.astype(np.float32)
    m = s64.view(np.uint64)
    tie = ((m & np.uint64((1 << 29) - 1)) == np.uint64(1 << 28)) & (s64 != 0)
    den = np.abs(s64) < 2.0 ** -126
    tt = s64[den] * 2.0 ** 149
    tie[den] = (tt - np.floor(tt)) == 0.5
    bad = int((q2.view(np.uint32) != ref.view(np.uint32))[~tie].sum())
    return bad, int(tie.sum())


if __name__ == '__main__':
    lo, hi = (int(sys.argv[1], 0), int(sys.argv[2], 0)) if len(sys.argv) > 2 else (0, 0x40400001)
    t = time.time()
    bad, ties = check(lo, hi)
    print('float bits %#x..%#x: mismatches %d, unresolved ties %d (%.1f s)' % (lo, hi, bad, ties, time.time() - t))
    sys.exit(1 if bad or ties else 0)
