#!/bin/bash
# r05 GPU call: one wave's dependent-chain latency per step for the MEA's lane-shift forms
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 tools/probe/dpp_latency | tee gpurun_out/dpp_latency.json
