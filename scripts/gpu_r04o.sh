#!/bin/bash
# Knob re-sweep on the round-4 plan: split thresholds, 128-tile threshold.
O=gpurun_out
timeout -k 10 900 python3 scripts/factor_breakdown.py --reps 10 --envs "ss32:PGO_STEP_SPLIT=32" "ss128:PGO_STEP_SPLIT=128" \
  "ss0:PGO_STEP_SPLIT=0" "fs32:PGO_FIRST_SPLIT=32" "fs128:PGO_FIRST_SPLIT=128" "bt2k:PGO_BIGTILE_MIN=2048" \
  "bt8k:PGO_BIGTILE_MIN=8192" "default2:PGO_DUMMY=2" > $O/r04o_ab.txt 2>&1 || { echo "ab failed"; tail -5 $O/r04o_ab.txt; exit 1; }
grep -v "^{" $O/r04o_ab.txt
