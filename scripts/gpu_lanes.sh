#!/bin/bash
# Lane/multi-rank parity tests, then bench lines for 1..3 lanes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_multi_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_lanes.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_lanes.log
[ $rc -eq 0 ] || exit $rc
for L in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --marginals 0 --lanes $L > gpurun_out/bench_lanes$L.log 2>&1
  rc=$?; echo "lanes $L rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' gpurun_out/bench_lanes$L.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['per_step'])"
done
