"""LOG_ADD's coefficient row from fma(d, 16M, -0.5) + 1.5 * 2^23 (round 6,
mlp_numerics.h) equals the truncating convert's row: every float within 4096
ulps of each multiple of 1/32 in [0, 7.5) (all row boundaries and their
neighbours) plus 2e7 random floats; tools/check_lookup_rows.py checks all
1.1e9 floats of [0, 7.5) (no mismatch)."""
import importlib.util
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tool():
    spec = importlib.util.spec_from_file_location('clr', os.path.join(ROOT, 'tools', 'check_lookup_rows.py'))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_rows_near_boundaries_and_sampled():
    t = _tool()
    edges = np.arange(0, 241, dtype=np.float32) / np.float32(32)   # every multiple of 1/32 up to 7.5
    eb = edges.view(np.uint32).astype(np.int64)
    near = (eb[:, None] + np.arange(-4096, 4097)[None, :]).ravel()
    near = near[(near >= 0) & (near < int(np.float32(7.5).view(np.uint32)))].astype(np.uint32)
    rng = np.random.default_rng(6)
    sample = rng.integers(0, int(np.float32(7.5).view(np.uint32)), 20_000_000, dtype=np.uint32)
    for bits in (np.unique(near), sample):
        _, cur, new = t.rows(bits)
        assert np.array_equal(cur, new)
