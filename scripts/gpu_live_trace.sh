#!/bin/bash
# The live re-solve under rocprofv3 --kernel-trace (checks that every dispatch of
# the re-planned solver is well-formed)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/lt
timeout -k 10 150 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/lt -o lt -- \
  python3 bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --live 2 --gicp 0 --search 0 --marginals 0 > gpurun_out/lt.log 2>&1
rc=$?; echo "live trace rc=$rc"; grep -v "^W2026\|^I2026" gpurun_out/lt.log | grep -iE "error|malformed|Traceback" | head -5
exit 0
