set -e -o pipefail
O=gpurun_out/r01h; mkdir -p $O
timeout -k 10 200 python -u tools/cold_posteriors.py > $O/cold.log 2>&1
MLP_SCRATCH_GB=24 timeout -k 10 200 python -u tools/cold_posteriors.py > $O/cold24.log 2>&1
timeout -k 10 300 tools/cli_time.sh 128 256 > $O/cli128.log 2>&1
cp gpurun_out/fam_128_256.err $O/cli128.err
timeout -k 10 400 tools/cli_time.sh 512 400 > $O/cli512.log 2>&1
cp gpurun_out/fam_512_400.err $O/cli512.err
