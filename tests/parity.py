"""Parity rules shared by the GPU tests.

Integer / index outputs (row pointers, column lists) and every value that does
not pass through the partition function are compared bit-exactly.  Values that
do (pid 0/1 merge, pid >= 3) carry the reference's x87 long double vs our
fp64 difference and are compared with |d| <= RTOL * max(|ref|, 1e-6); an entry
present on one side only is accepted iff its value is within RTOL of the 0.01
cutoff (CPNP/SparseMatrix.h:14).
"""
import numpy as np

RTOL = 1e-4
CUTOFF = np.float32(0.01)


def dense_rows(rp, cols, vals):
    out = {}
    for i in range(1, len(rp) - 1):
        for e in range(rp[i], rp[i + 1]):
            out[(i, int(cols[e]))] = float(vals[e])
    return out


def csr_equal(ref, ours, what=''):
    np.testing.assert_array_equal(np.asarray(ours[0]), np.asarray(ref[0]), err_msg=f'{what} rowptr')
    np.testing.assert_array_equal(np.asarray(ours[1]), np.asarray(ref[1]), err_msg=f'{what} cols')
    np.testing.assert_array_equal(np.asarray(ours[2], np.float32), np.asarray(ref[2], np.float32),
                                  err_msg=f'{what} vals')


def csr_close(ref, ours, rtol=RTOL, what=''):
    """Returns (max relative error, cutoff flips); asserts the rule."""
    R = dense_rows(*ref)
    O = dense_rows(*ours)
    worst = 0.0
    flips = 0
    for k in set(R) | set(O):
        if k in R and k in O:
            r, o = R[k], O[k]
            err = abs(o - r) / max(abs(r), 1e-6)
            worst = max(worst, err)
            assert err <= rtol, f'{what} cell {k}: ref {r!r} ours {o!r} rel {err:.3g}'
        else:
            v = R.get(k, O.get(k))
            flips += 1
            assert abs(v - float(CUTOFF)) <= rtol * float(CUTOFF) * 10, \
                f'{what} cell {k} only on one side with value {v!r} (not at the cutoff)'
    return worst, flips


def close_scalar(ref, ours, rtol=RTOL):
    return abs(float(ours) - float(ref)) <= rtol * max(abs(float(ref)), 1e-6)
