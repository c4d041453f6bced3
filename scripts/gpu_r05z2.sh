#!/bin/bash
# Round 5, after the kernel changes: a replay sweep of the schedule knobs
# (scripts/factor_breakdown.py, C3, 1 / 3 lanes), the default run twice as
# the noise reference.
set -o pipefail
O=gpurun_out
timeout -k 10 900 python3 scripts/factor_breakdown.py --config C3 --lanes 1 3 --envs \
  "base2:PGO_VEC_FUSE=1" "sideprio:PGO_SIDE_PRIORITY=1" "fs32:PGO_FIRST_SPLIT=32" "fs128:PGO_FIRST_SPLIT=128" \
  "fsoff:PGO_FIRST_SPLIT=1000000" "ss64:PGO_STEP_SPLIT=64" "unroll2:PGO_ASM_UNROLL=2" "far:PGO_FAR=1" "base3:PGO_VEC_FUSE=1" \
  > $O/r05z2_sweep.txt 2>&1 || { tail -20 $O/r05z2_sweep.txt; exit 1; }
tail -1 $O/r05z2_sweep.txt
