#!/bin/bash
# Per-level split of a factorisation replay (1 and 3 lambda lanes) on the GPU
# box: rocprofv3 kernel traces of scripts/replay_trace.py summarised by
# scripts/level_summary.py, plus a quick default bench.  Usage (from the repo
# root on the box): bash scripts/gpu_levels.sh TAG
set -o pipefail
TAG=${1:-cur}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/levels_$TAG
mkdir -p $OUT
for L in 1 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $OUT/t$L -o t -- \
    python3 scripts/replay_trace.py --lanes $L --reps 2 > $OUT/replay_l$L.log 2>&1 || exit 1
  f=$(find $OUT/t$L -name "*kernel_trace.csv" | head -1)
  python3 scripts/level_summary.py "$f" > $OUT/levels_l$L.txt || exit 1
  gzip -f "$f"
  echo "lanes $L"; tail -40 $OUT/levels_l$L.txt
done
