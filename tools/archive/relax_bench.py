"""Time one relaxation round at C3 (or N L) from the same posterior sparse set,
per relaxation path (MLP_RELAX = default / tasks), e.g. on the GPU box:
    python tools/relax_bench.py [N L [modes]]
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
from mlprobs_amd import synth, engine  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    L = int(sys.argv[2]) if len(sys.argv) > 2 else 400
    modes = sys.argv[3].split(',') if len(sys.argv) > 3 else ['default']
    seqs = [s for _, s in synth.family(n, L, 0.7, seed=11)]
    fam = engine.Family(seqs)
    fam.posteriors(0, float(os.environ.get("MLP_DELTA", "0.132548")))
    csr = [a.copy() for a in fam.export()]
    print(f'n={n} L={L} nnz={len(csr[2])}', flush=True)
    for mode in modes:
        if mode == 'default':
            os.environ.pop('MLP_RELAX', None)
        else:
            os.environ['MLP_RELAX'] = mode
        for rep in range(2):
            fam.import_csr(*csr)
            fam.synchronize()
            fam.profile(True)
            t = time.perf_counter()
            fam.relax(1)
            fam.synchronize()
            dt = time.perf_counter() - t
            kt = fam.kernel_times()
            print(f'{mode} rep{rep}: {dt:.3f} s  relax kernel {kt["relax"]["ms"]:.1f} ms  '
                  f'pack/transpose {kt["transpose"]["ms"]:.1f} ms  nnz out {fam.export()[2].size}', flush=True)


if __name__ == '__main__':
    main()
