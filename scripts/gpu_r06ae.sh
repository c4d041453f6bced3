#!/bin/bash
# Round 6: the schedule knobs re-swept on this round's kernels (factorisation
# replays at 1 / 3 lanes, two rounds): 128-tile threshold, look-ahead front
# height, step / first-panel split thresholds.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ae
mkdir -p $O
for k in 1 2; do
  timeout -k 10 900 python3 scripts/factor_breakdown.py --config C3 --lanes 1 3 --reps 8 \
    --envs "big2048:PGO_BIGTILE_MIN=2048" "big8192:PGO_BIGTILE_MIN=8192" "la256:PGO_LOOKAHEAD_M=256" "la1024:PGO_LOOKAHEAD_M=1024" \
           "split32:PGO_STEP_SPLIT=32" "split128:PGO_STEP_SPLIT=128" "first32:PGO_FIRST_SPLIT=32" "first128:PGO_FIRST_SPLIT=128" > $O/replay$k.txt 2>&1 || exit 1
  tail -1 $O/replay$k.txt
done
echo done
