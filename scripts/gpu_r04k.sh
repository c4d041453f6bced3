#!/bin/bash
# Look-ahead height threshold sweep (PGO_LOOKAHEAD_M; default 2048), replays.
O=gpurun_out
timeout -k 10 900 python3 scripts/factor_breakdown.py --reps 10 --envs "la1024:PGO_LOOKAHEAD_M=1024" \
  "la512:PGO_LOOKAHEAD_M=512" "la256:PGO_LOOKAHEAD_M=256" "la128:PGO_LOOKAHEAD_M=128" "la64:PGO_LOOKAHEAD_M=64" \
  "default2:PGO_DUMMY=2" "la512b:PGO_LOOKAHEAD_M=512" "la256b:PGO_LOOKAHEAD_M=256" > $O/r04k_ab.txt 2>&1 || { echo "ab failed"; tail -5 $O/r04k_ab.txt; exit 1; }
grep -v "^{" $O/r04k_ab.txt
