"""Exhaustive check of LOG_ADD's coefficient-row index (mlp_numerics.h,
mlp_log_add_t): on every float d in [0, 7.5) the row the sweeps read,
(bits(fma(d, 16M, -0.5) + 1.5 * 2^23) & 0xf0), equals the one of the
truncating convert it replaced, (int)fl(d * 16M) & 0xf0, 16M = 0x1.fffffep4.
(Above 7.5 the select returns hi whatever the row; the mask keeps the read
inside the table.)  The fma is emulated exactly: d * 16M is exact in double,
d * 16M - 0.5 too where it matters (d * 16M >= 2^-6; below, both rows are 0),
and each float rounding is one cast from an exact double.  ~35 s on 1.1e9 floats.

    python tools/check_lookup_rows.py [lo_bits hi_bits]
"""
import sys

import numpy as np

K = np.float32(float.fromhex('0x1.fffffep4'))
C = np.float64(12582912.0)  # 1.5 * 2^23


def rows(bits):
    d = bits.view(np.float32)
    p = d.astype(np.float64) * np.float64(K)  # exact (24 x 24 bits)
    cur = np.trunc(p.astype(np.float32)).astype(np.int64) & 0xf0
    t = (p - 0.5).astype(np.float32)  # RN32(d * 16M - 0.5)
    u = (t.astype(np.float64) + C).astype(np.float32)  # RN32(t + C): the sum is exact
    new = u.view(np.int32).astype(np.int64) & 0xf0
    return d, cur, new


def main():
    end = int(np.frombuffer(np.float32(7.5).tobytes(), np.uint32)[0])
    lo, hi = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (0, end)
    bad = 0
    for a in range(lo, hi, 1 << 24):
        d, cur, new = rows(np.arange(a, min(a + (1 << 24), hi), dtype=np.uint32))
        m = np.nonzero(cur != new)[0]
        bad += len(m)
        if len(m):
            print('mismatch at', d[m[:5]], cur[m[:5]], new[m[:5]])
    print(f'checked {hi - lo} floats, {bad} mismatches')
    return 1 if bad else 0


if __name__ == '__main__':
    sys.exit(main())
