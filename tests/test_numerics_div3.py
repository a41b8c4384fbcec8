"""mlp_div3 (mlp_numerics.h, the merge's x / 3 by FMA correction) against the
IEEE quotient: every float of the denormal range and of the binades
[0.5, 1) and [1, 3], and a random sample of the rest of [0, 3].  The whole
range is checked by tools/check_div3.py (1.08e9 values, no mismatch)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tools'))
import check_div3  # noqa: E402


def test_div3_denormals():
    assert check_div3.check(0, 0x00800000) == (0, 0)


def test_div3_binades_near_one():
    assert check_div3.check(0x3f000000, 0x40400001) == (0, 0)


def test_div3_random_sample():
    rng = np.random.default_rng(7)
    bits = rng.integers(0, 0x40400001, size=1 << 22, dtype=np.uint32)
    assert check_div3.check_values(bits.view(np.float32)) == (0, 0)
