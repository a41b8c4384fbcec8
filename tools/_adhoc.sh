set -e -o pipefail
O=gpurun_out/r01y4; mkdir -p $O
timeout -k 10 300 python -u tools/pf_check4.py > $O/pf4.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
