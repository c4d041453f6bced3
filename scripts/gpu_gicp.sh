# GICP: GPU tests, the batch bench and a kernel-trace summary
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gicp.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/gicp_test.log 2>&1 &&
timeout -k 10 300 python -u scripts/gicp_only.py ${GICP_B:-1024} > gpurun_out/gicp_bench.json 2> gpurun_out/gicp_bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/gicp_prof -o run -- python3 scripts/gicp_only.py ${GICP_B:-1024} > gpurun_out/gicp_prof.log 2>&1
