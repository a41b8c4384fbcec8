#!/bin/bash
# Run GPU steps in order on the box, each under its own time limit; stop at
# the first step that times out, aborts or faults (exit status other than 0
# or 1).  Usage: tools/gpu_steps.sh 'name|seconds|command' ...
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  echo "[step $name] $(date +%T) start"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.txt" 2>&1
  rc=$?
  echo "[step $name] $(date +%T) rc $rc"; tail -3 "gpurun_out/$name.txt"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
done
