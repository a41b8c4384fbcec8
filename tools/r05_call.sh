#!/bin/bash
# round-5 working call: forward sweep A/B (transition constants in VGPRs at 4 waves; 4 waves alone)
set -o pipefail
export TMPDIR=/tmp
bash tools/variant_bench.sh base vc4 fw4 base
