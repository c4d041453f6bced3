#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for q in 4 8; do for l in 1 2; do
GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --marginals 0 --search 0 --lanes $l > gpurun_out/bench_nd_q${q}_l${l}.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
grep '^{' gpurun_out/bench_nd_q${q}_l${l}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('q$q l$l', d['value'], d['ms_per_step'], d['per_step']['lambda_rounds'])"
done; done
