#!/bin/bash
# bench at 2/3/4 lambda lanes (no side lines)
set -o pipefail
mkdir -p gpurun_out
for l in 2 3 4; do
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --marginals 0 --search 0 --live 0 --gicp 0 --lanes $l > gpurun_out/bench_lanes$l.log 2>&1
  rc=$?; [ $rc -eq 0 ] || exit $rc
  grep '^{' gpurun_out/bench_lanes$l.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lanes $l', d['value'], d['ms_per_step'], d['per_step']['lambda_rounds'], d['per_step']['solves_rank0'])"
done
