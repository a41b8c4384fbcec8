#!/bin/bash
# One GPU-box call: the -m gpu suite, smoke(), then the bench line with its
# rocprofv3 kernel statistics from the same command.
#   tools/gpu_round.sh TAG [pytest args...] -> gpurun_out/TAG/{gputest.log,smoke.log,bench.json,stats/}
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-round}; shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" \
    > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -3 $O/gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tools/gpu_bench.sh $TAG || exit 1
echo done
