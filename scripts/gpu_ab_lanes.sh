#!/bin/bash
# A/B of the lambda-lane count (adaptive rounds): quick C3 bench, 2 runs each
set -o pipefail
mkdir -p gpurun_out
for lanes in ${LANES:-2 3 2 3}; do
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --live 0 --gicp 0 --search 0 --marginals 0 \
    --lanes $lanes > gpurun_out/ab_lanes.log 2>&1 || exit $?
  grep '^{' gpurun_out/ab_lanes.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['per_step']; print('lanes $lanes', round(d['value'],3), p['lambda_rounds'], p['solves_rank0'])" | tee -a gpurun_out/ab_lanes.txt
done
