set -e -o pipefail
bash tools/pmc_run.sh gpurun_out/pmc_r01n "--steps 1 --warmup 0 --no-cpu --no-e2e --no-qp --relax 0"
