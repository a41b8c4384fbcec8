"""Build experiment copies of libmlpgpu (lib/libmlpgpu_<name>.so, loaded with
MLP_LIB_VARIANT=<name>; never the default) from name=DEFINE[,DEFINE...] args:
    python tools/build_variants.py w5=MLP_SWEEP_WAVES=5 nochain=MLP_EXP_NOCHAIN
    python tools/build_variants.py --rev base=HEAD     (the sources of a git revision)
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


def from_rev(spec):
    """name=REV: the library as built from git revision REV's sources."""
    import subprocess
    import tempfile
    name, rev = spec.split('=', 1)
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
    tmp = tempfile.mkdtemp(prefix=f'mlp_rev_{name}_')
    arch = subprocess.run(['git', '-C', root, 'archive', rev, 'mlprobs_amd/csrc', 'include'], check=True,
                          capture_output=True).stdout
    subprocess.run(['tar', '-x', '-C', tmp], input=arch, check=True)
    b.build(variant=name, src_root=tmp)
    return name


if __name__ == '__main__':
    args = sys.argv[1:]
    if args and args[0] == '--rev':
        for spec in args[1:]:
            print('built', from_rev(spec))
        sys.exit(0)
    with ThreadPoolExecutor(4) as ex:
        for n in ex.map(one, args):
            print('built', n)
