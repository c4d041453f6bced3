#!/bin/bash
# Kernel trace of one graph-mode C3 bench step (per-kernel timeline of the
# captured factor+solve; scripts/steps.py reads it).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g
timeout -k 10 400 rocprofv3 --kernel-trace -T -f csv -d gpurun_out/g -o c3 -- \
  python3 bench.py --config C3 --steps 1 --warmup 1 --no-cpu-baseline --live 0 --gicp 0 --search 0 --marginals 0 > gpurun_out/g.log 2>&1
rc=$?; echo "gtrace rc=$rc"; [ $rc -eq 0 ] || exit $rc
find gpurun_out/g -name "*kernel_trace.csv" -exec gzip -f {} \;
