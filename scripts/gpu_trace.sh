#!/bin/bash
# Kernel-trace stats of one bench step (quick profile, no PMC).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/trace_${TAG:-q}
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT -o run -- \
  python3 bench.py --config ${CONFIG:-C3} --steps 1 --warmup 0 --no-cpu-baseline --no-graphs ${BENCH_ARGS:-} > $OUT/bench.log 2>&1
rc=$?; echo "trace rc=$rc"
find $OUT -name "*kernel_trace.csv" -exec gzip -f {} \;
exit $rc
