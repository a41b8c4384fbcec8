"""Dense-block MFMA relaxation vs k_relax_tile at C3 (GPU box):
    python tools/relax_mfma_eval.py [N L] > gpurun_out/mfma_eval.json
One exact consistency round (k_relax_tile, all pairs) is timed first, then the
dense 16x16 block MFMA variant (relax_mfma.hip) on 32 x 32 output pairs of the same
store; its time is extrapolated to every pair.  SURVEY.md section 7 step 6."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mlprobs_amd import synth  # noqa: E402
from mlprobs_amd.engine import Family  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
L = int(sys.argv[2]) if len(sys.argv) > 2 else 400
os.environ.setdefault('MLP_SCRATCH_GB', '32')
fam = Family([s for _, s in synth.family(n, L, 0.7, seed=11)])
fam.posteriors(0, 0.132548)
k = int(os.environ.get('MFMA_SIDE', '32'))   # k x k output pairs: enough workgroups to fill the device
xs = list(range(k))
ys = list(range(n // 2, n // 2 + k))
t0 = time.perf_counter()
r = fam.relax_blockmfma_eval(xs, ys)
wall = time.perf_counter() - t0
P = n * (n - 1) // 2
peak_macs = 157.3e12 / 2   # fp32 MFMA (MI355X_MICROARCH.md)
out = {'family': f'{n}x{L} s=0.7 seed 11', 'mfma': r, 'host_wall_s': wall,
       'mfma_dense_mac_per_s': r['dense_macs'] / r['seconds'],
       'mfma_util': r['dense_macs'] / r['seconds'] / peak_macs,
       'mfma_round_s_extrapolated': r['seconds'] * P / r['outputs']}
# the exact kernel on the whole family, same store
fam.profile(True)
t0 = time.perf_counter()
fam.relax(1)
fam.synchronize()
out['tile_round_s'] = time.perf_counter() - t0
kt = fam.kernel_times()
out['tile_kernel_ms'] = {k: v['ms'] for k, v in kt.items() if v['launches']}
out['tile_per_output_ms'] = out['tile_kernel_ms'].get('relax', 0) / P
out['mfma_per_output_ms'] = r['seconds'] * 1e3 / r['outputs']
print(json.dumps(out, indent=1))
fam.close()
