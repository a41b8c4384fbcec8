"""CPU-side checks of the C ABI library: it builds for gfx950, loads, and
exports every symbol include/mlpgpu.h declares (no compute without a GPU)."""
import ctypes
import os
import re

from mlprobs_amd import build as mbuild
from mlprobs_amd import engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    txt = open(os.path.join(ROOT, 'include', 'mlpgpu.h')).read()
    return sorted(set(re.findall(r'\b(mlp_[a-z_]+)\s*\(', txt)))


def test_build_and_symbols():
    path = mbuild.build()
    assert os.path.exists(path)
    L = ctypes.CDLL(path)
    for name in declared():
        assert hasattr(L, name), name
    assert sorted(engine.EXPORTED) == declared()


def test_gfx950_code_object():
    data = open(mbuild.build(), 'rb').read()
    assert b'gfx950' in data
