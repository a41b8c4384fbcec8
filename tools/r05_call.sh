#!/bin/bash
# round-5: the GPU suite on the current tree
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.txt 2>&1; rc=$?
tail -5 $O/gputest.txt
exit $rc
