#!/bin/bash
# Development loop on the GPU box: selected parity tests, a graph-mode bench
# line, then a kernel-trace of one eager bench step.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x -k "${PYTEST_K:-cholesky or lm_parity or c3 or smoke}" > gpurun_out/pytest_dev.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_dev.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_dev.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_dev.log | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
TAG=${TAG:-dev} bash scripts/gpu_trace.sh
