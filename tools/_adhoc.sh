set -e -o pipefail
O=gpurun_out/r01e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_cli_gpu.py -m gpu -v --timeout 120 --timeout-method thread -k edge > $O/pytest.log 2>&1 || true
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
