#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_search.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_search.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_search.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --marginals 0 > gpurun_out/bench_search.log 2>&1
rc=$?; echo "bench rc=$rc"
grep '^{' gpurun_out/bench_search.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['closest_keyframe'])"
exit $rc
