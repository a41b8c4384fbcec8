"""Build libmlpgpu.so (HIP kernels for gfx950 + C-ABI host runtime) in-tree.

    python -m mlprobs_amd.build

hipcc flags: -ffp-contract=off keeps every float operation unfused so the
DP reproduces the reference's scalar-SSE rounding sequence (no FMA); no
fast-math; fp32 division / sqrt stay correctly rounded (hipcc default).
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, 'csrc')
LIBDIR = os.path.join(HERE, 'lib')
LIB = os.path.join(LIBDIR, 'libmlpgpu.so')
SOURCES = ['posterior.hip', 'totals.hip', 'viterbi.hip', 'relax.hip', 'relax_mfma.hip', 'profile.hip', 'mlp_knobs.cpp',
           'mlp_context.cpp', 'mlp_planner.cpp', 'mlp_posteriors.cpp', 'mlp_profile_rt.cpp', 'mlp_shards.cpp',
           'mlp_relax_rt.cpp', 'host_backend.cpp']
HEADERS = ['mlp_kernels.h', 'mlp_numerics.h', 'mlp_chain.h', 'mlp_params_default.inc', 'mlp_params_qp.inc',
           'host_backend.h', 'mlp_runtime.h', 'mlp_knobs.h']
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
# -fno-slp-vectorize: the SLP pass packs adjacent f32 adds/multiplies of the
# DP cell updates into v_pk_*_f32 and pays for it in register moves; without
# it the forward/backward sweeps run 4% faster at C3 (same results).
FLAGS = ['--offload-arch=gfx950', '-O3', '-ffp-contract=off', '-fno-fast-math', '-fno-slp-vectorize', '-fPIC',
         '-std=c++17', '-Wno-unused-result', '-Wno-unused-value']


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(ROOT, 'include', 'mlpgpu.h')]
    return any(os.path.getmtime(d) > t for d in deps)


def variant_path(name):
    return os.path.join(LIBDIR, f'libmlpgpu_{name}.so')


def build(force=False, verbose=False, variant=None, defines=(), src_root=None):
    """Build the library; `variant` builds an experiment copy
    lib/libmlpgpu_<variant>.so with extra -D defines (loaded when
    MLP_LIB_VARIANT=<variant>; never the default), optionally from another
    source tree `src_root` (its csrc/ and include/, e.g. a git revision
    exported by tools/build_variants.py --rev, for same-call A/Bs)."""
    out = variant_path(variant) if variant else LIB
    csrc = os.path.join(src_root, 'mlprobs_amd', 'csrc') if src_root else CSRC
    inc = os.path.join(src_root, 'include') if src_root else os.path.join(ROOT, 'include')
    if not variant and not force and not _stale():
        return LIB
    os.makedirs(LIBDIR, exist_ok=True)
    extra = os.environ.get('MLP_EXTRA_FLAGS', '').split() if variant else []  # experiment copies only
    # one object per source, compiled concurrently (the kernels are
    # independent translation units), then one link
    objdir = os.path.join(HERE, '_build', variant or 'default')
    os.makedirs(objdir, exist_ok=True)
    base = [HIPCC] + FLAGS + extra + ['-D' + d for d in defines] + ['-I', inc]
    procs, objs = [], []
    for f in SOURCES:
        obj = os.path.join(objdir, f + '.o')
        objs.append(obj)
        cmd = base + ['-c', os.path.join(csrc, f), '-o', obj]
        if verbose:
            print(' '.join(cmd))
        procs.append(subprocess.Popen(cmd))
    if any(p.wait() != 0 for p in procs):
        raise subprocess.CalledProcessError(1, 'hipcc -c')
    cmd = [HIPCC, '--offload-arch=gfx950', '-shared', '-fPIC'] + objs + ['-lrccl', '-o', out + '.tmp']
    if verbose:
        print(' '.join(cmd))
    subprocess.check_call(cmd)
    os.replace(out + '.tmp', out)
    return out


if __name__ == '__main__':
    args = sys.argv[1:]
    var = args[args.index('--variant') + 1] if '--variant' in args else None
    defs = [a[2:] for a in args if a.startswith('-D')]
    print(build(force='--force' in args, verbose=True, variant=var, defines=defs))
