#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprof kernel stats.
# Usage (from the repo root on the box): tools/gpu_check.sh [tag]
set -e -o pipefail
export TMPDIR=/tmp
TAG=${1:-check}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python -u bench.py --relax 1 > $O/bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o stats -- python3 bench.py --steps 2 --warmup 1 --no-cpu --relax 1 > $O/stats.log 2>&1
echo done
