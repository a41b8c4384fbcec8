"""Debug helper (GPU box): the posterior stage on one golden pair, printing
the error instead of raising (tests/golden pair fixtures)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'tests'))
from mlprobs_amd.engine import Family  # noqa: E402
from goldens import load_pair  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else 'div30'
pid = int(sys.argv[2]) if len(sys.argv) > 2 else 0
d = load_pair(name)
fam = Family([d['s1'], d['s2']])
try:
    fam.posteriors(pid, float(d['delta']))
    print('ok', fam.results()[0][:1], flush=True)
except Exception as e:  # noqa: BLE001
    print('error', e, flush=True)
    sys.exit(3)
