#!/bin/bash
# Tile-assembly A/B: children's loads one vs two children in flight
# (PGO_ASM_UNROLL), bitwise check of the optimize under both, then replays.
O=gpurun_out
for v in 1 2; do
  PGO_ASM_UNROLL=$v timeout -k 10 200 python3 scripts/bitwise_env_check.py --lanes 3 || { echo "check $v failed"; exit 1; }
done
timeout -k 10 400 python3 scripts/factor_breakdown.py --reps 10 --envs "u1:PGO_ASM_UNROLL=1" "u2:PGO_ASM_UNROLL=2" \
  "u1b:PGO_ASM_UNROLL=1" "u2b:PGO_ASM_UNROLL=2" > $O/r04i_ab.txt 2>&1 || { echo "ab failed"; exit 1; }
tail -1 $O/r04i_ab.txt
