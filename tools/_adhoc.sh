set -e -o pipefail
O=gpurun_out/r01f4; mkdir -p $O
for r in 1 2; do
  MLP_PROFILE_TIMES=1 timeout -k 10 300 bash tools/qp_cli_time.sh 512 400 > /dev/null 2>&1; cp gpurun_out/qpfam_512_400.time $O/qp$r.time
done
timeout -k 10 900 python -u -m pytest tests/test_cli_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_cli.log 2>&1
