set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gicp.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/gicp_test.log 2>&1
