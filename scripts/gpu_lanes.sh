#!/bin/bash
# Batched lambda lanes: lane tests, then the full GPU suite, then bench at 1/2/3 lanes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_multi_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "lanes or lane_count" > gpurun_out/pytest_lanes.log 2>&1
rc=$?; echo "lane tests rc=$rc"; tail -3 gpurun_out/pytest_lanes.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_iter.log; [ $rc -eq 0 ] || exit $rc
for l in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --marginals 0 --search 0 --lanes $l > gpurun_out/bench_lanes$l.log 2>&1
  rc=$?; [ $rc -eq 0 ] || exit $rc
  grep '^{' gpurun_out/bench_lanes$l.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lanes $l', d['value'], d['ms_per_step'], d['per_step']['lambda_rounds'])"
done
