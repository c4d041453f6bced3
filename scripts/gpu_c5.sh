#!/bin/bash
# C5 (1M poses / 5M edges) on one MI355X: the full-size parity test, then one
# bench step with the per-launch profile and a rocprofv3 kernel-stats pass.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k c5 -x -v --timeout 380 --timeout-method thread \
  > gpurun_out/c5_test.log 2>&1
rc=$?; echo "c5 test rc=$rc"; tail -3 gpurun_out/c5_test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --config C5 --steps 1 --warmup 0 --no-cpu-baseline --marginals 0 --search 0 \
  --profile-every 16 > gpurun_out/c5_bench.log 2>&1
rc=$?; echo "c5 bench rc=$rc"; tail -c 400 gpurun_out/c5_bench.log
