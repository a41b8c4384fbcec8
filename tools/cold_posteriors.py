"""Cold vs warm posterior-stage timing (first call includes allocation and
code-object loading): python tools/cold_posteriors.py [N L]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
from mlprobs_amd import synth, engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
L = int(sys.argv[2]) if len(sys.argv) > 2 else 400
seqs = [s for _, s in synth.family(n, L, 0.7, seed=11)]
t = time.perf_counter()
fam = engine.Family(seqs)
fam.synchronize()
print(f'create+load {time.perf_counter() - t:.3f} s', flush=True)
for rep in range(3):
    t = time.perf_counter()
    fam.posteriors(0, 0.132548)
    fam.synchronize()
    print(f'posteriors rep{rep} {time.perf_counter() - t:.3f} s', flush=True)
