set -e -o pipefail
O=gpurun_out/r01f2; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 bash tools/qp_cli_time.sh 512 400 > /dev/null 2>&1; cp gpurun_out/qpfam_512_400.time $O/qp$r.time
  timeout -k 10 300 bash tools/cli_time.sh 512 400 > /dev/null 2>&1; cp gpurun_out/fam_512_400.time $O/cp$r.time
done
