#!/bin/bash
# Quick GPU check with tight limits: all GPU parity tests, one bench line, and
# (GTRACE=1) a kernel trace of a graph-mode step.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 ${T_TEST:-300} python -m pytest tests -m gpu -q -x > gpurun_out/pytest_quick.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_quick.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 ${T_BENCH:-240} python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_quick.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_quick.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
[ -z "$GTRACE" ] || bash scripts/gpu_gtrace.sh
