#!/bin/bash
# Lanes vs hardware queues per process (GPU_MAX_HW_QUEUES), eager launches.
set -o pipefail
mkdir -p gpurun_out
for Q in 4 8; do
for L in 1 2; do
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --marginals 0 --lanes $L --no-graphs > gpurun_out/bench_e_q${Q}_l$L.log 2>&1
  rc=$?; echo "eager Q $Q lanes $L rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' gpurun_out/bench_e_q${Q}_l$L.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['per_step']; print(round(d['value'],2), round(d['ms_per_step'],1), p['lambda_rounds'], round(p['ms_solve'],1))"
done
done
