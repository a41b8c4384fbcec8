set -e -o pipefail
bash tools/relax_pmc.sh gpurun_out/rpmc2
