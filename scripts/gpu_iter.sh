#!/bin/bash
# Iteration check: all GPU parity tests, one default bench line, a graph-mode
# kernel trace (scripts/steps.py reads gpurun_out/g/).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 ${T_TEST:-400} python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_iter.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --marginals 0 --search 0 ${BENCH_ARGS:-} > gpurun_out/bench_iter.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
grep '^{' gpurun_out/bench_iter.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['per_step']['lm_tries'], d['per_step']['final_error'])"
[ -z "$GTRACE" ] || bash scripts/gpu_gtrace.sh
