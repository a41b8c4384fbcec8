#!/bin/bash
# r05 GPU call: the whole GPU suite + smoke at HEAD
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gputest.txt 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1
rc=$?; tail -3 $O/gputest.txt; cat $O/smoke.txt | tail -2; exit $rc
