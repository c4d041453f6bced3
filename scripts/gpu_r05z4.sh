#!/bin/bash
# k_step's first diagonal tile with its task and front scalars as kernel
# arguments (PGO_DIAG_META, default 1; 0: loaded through the task list):
# bitwise C2 / C3, root-level step stamps, replay A/B (alternating).
set -o pipefail
O=gpurun_out
: > $O/r05z4_bitwise.txt
for v in 1 0; do
  PGO_DIAG_META=$v timeout -k 10 200 python3 scripts/bitwise_env_check.py --config C3 --lanes 3 >> $O/r05z4_bitwise.txt 2>&1 || { tail -20 $O/r05z4_bitwise.txt; exit 1; }
done
timeout -k 10 200 python3 scripts/bitwise_env_check.py --config C2 --lanes 1 >> $O/r05z4_bitwise.txt 2>&1 || { tail -20 $O/r05z4_bitwise.txt; exit 1; }
grep final $O/r05z4_bitwise.txt
TAG=meta1 PGO_DIAG_META=1 bash scripts/gpu_stamps.sh > $O/r05z4_stamps1.txt || exit 1
TAG=meta0 PGO_DIAG_META=0 bash scripts/gpu_stamps.sh > $O/r05z4_stamps0.txt || exit 1
tail -4 $O/r05z4_stamps1.txt; tail -4 $O/r05z4_stamps0.txt
timeout -k 10 600 python3 scripts/factor_breakdown.py --config C3 --lanes 1 3 --envs "m0:PGO_DIAG_META=0" "m1:PGO_DIAG_META=1" "m0b:PGO_DIAG_META=0" "m1b:PGO_DIAG_META=1" > $O/r05z4_replay.txt 2>&1 || { tail -20 $O/r05z4_replay.txt; exit 1; }
tail -1 $O/r05z4_replay.txt
