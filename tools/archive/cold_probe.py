"""Cold vs warm posterior stage in one fresh process (GPU box):
    python tools/cold_probe.py N L [scratch_gb]
Prints the first (cold) and two warm mlp_posteriors times with per-kernel
device times, so a slow first call can be split into kernel time and the
rest (allocation, host waits)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
n, L = int(sys.argv[1]), int(sys.argv[2])
if len(sys.argv) > 3:
    os.environ['MLP_SCRATCH_GB'] = sys.argv[3]
from mlprobs_amd import synth  # noqa: E402
from mlprobs_amd.engine import Family  # noqa: E402

t0 = time.perf_counter()
fam = Family([s for _, s in synth.family(n, L, 0.7, seed=11)])
t_init = time.perf_counter() - t0
out = {'n': n, 'L': L, 'scratch_gb': os.environ.get('MLP_SCRATCH_GB'), 'init_s': t_init, 'calls': []}
for k in range(3):
    fam.profile(True)
    t0 = time.perf_counter()
    fam.posteriors(0, 0.132548)
    fam.synchronize()
    dt = time.perf_counter() - t0
    kt = fam.kernel_times()
    out['calls'].append({'s': dt, 'kernels_ms': {a: round(b['ms'], 1) for a, b in kt.items() if b['launches']},
                         'launches': {a: b['launches'] for a, b in kt.items() if b['launches']}})
for k in range(2):
    fam.profile(True)
    t0 = time.perf_counter()
    fam.relax(1) if k == 0 else None
    fam.synchronize()
    if k == 0:
        kt = fam.kernel_times()
        out['relax_s'] = time.perf_counter() - t0
        out['relax_kernels_ms'] = {a: round(b['ms'], 1) for a, b in kt.items() if b['launches']}
out["chain_rows"] = os.environ.get("MLP_CHAIN_ROWS")
out["two"] = os.environ.get("MLP_TWO")
print(json.dumps(out))
fam.close()
