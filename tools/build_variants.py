"""Build experiment copies of libmlpgpu (lib/libmlpgpu_<name>.so, loaded with
MLP_LIB_VARIANT=<name>; never the default) from name=DEFINE[,DEFINE...] args:
    python tools/build_variants.py w5=MLP_SWEEP_WAVES=5 nochain=MLP_EXP_NOCHAIN
"""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
from mlprobs_amd import build as b  # noqa: E402


def one(spec):
    name, defs = spec.split('=', 1)
    b.build(variant=name, defines=[d for d in defs.split(',') if d])
    return name


if __name__ == '__main__':
    with ThreadPoolExecutor(4) as ex:
        for n in ex.map(one, sys.argv[1:]):
            print('built', n)
