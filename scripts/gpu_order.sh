#!/bin/bash
# Nested dissection vs AMD: GPU parity tests (default = ND), bench with each ordering.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 ${T_TEST:-400} python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_order.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_order.log
[ $rc -eq 0 ] || exit $rc
for o in nd amd; do
  timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --marginals 0 --search 0 --ordering $o > gpurun_out/bench_order_$o.log 2>&1
  rc=$?; echo "bench $o rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' gpurun_out/bench_order_$o.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['per_step']['lm_tries'], d['per_step']['final_error'], d['roofline']['achieved'])"
done
