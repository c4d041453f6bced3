#!/bin/bash
# Small-front classes on a fourth side stream (PGO_WAVE_STREAMS=1): bitwise check, replay A/B.
O=gpurun_out
for v in 0 1; do
  PGO_WAVE_STREAMS=$v timeout -k 10 200 python3 scripts/bitwise_env_check.py --lanes 3 || { echo "check $v failed"; exit 1; }
done
timeout -k 10 400 python3 scripts/factor_breakdown.py --reps 10 --envs "ws:PGO_WAVE_STREAMS=1" "default2:PGO_DUMMY=2" \
  "wsb:PGO_WAVE_STREAMS=1" > $O/r04s_ab.txt 2>&1 || { echo "ab failed"; tail -5 $O/r04s_ab.txt; exit 1; }
grep -v "^{" $O/r04s_ab.txt
