#!/bin/bash
# k_step's payload hand-off (PGO_NAN_HANDOFF, default on): bitwise C2 / C3 against
# the flag protocol's known results, replay A/B against PGO_NAN_HANDOFF=0, the
# bench's k_step line, and the GPU tests.
set -o pipefail
O=gpurun_out
timeout -k 10 200 python3 scripts/bitwise_env_check.py --config C3 --lanes 3 > $O/r05w_bitwise.txt 2>&1 || { tail -20 $O/r05w_bitwise.txt; exit 1; }
PGO_NAN_HANDOFF=0 timeout -k 10 200 python3 scripts/bitwise_env_check.py --config C3 --lanes 3 >> $O/r05w_bitwise.txt 2>&1 || { tail -20 $O/r05w_bitwise.txt; exit 1; }
timeout -k 10 200 python3 scripts/bitwise_env_check.py --config C2 --lanes 1 >> $O/r05w_bitwise.txt 2>&1 || { tail -20 $O/r05w_bitwise.txt; exit 1; }
grep -E "final" $O/r05w_bitwise.txt
timeout -k 10 400 python3 scripts/factor_breakdown.py --config C3 --lanes 1 3 --envs "flag:PGO_NAN_HANDOFF=0" "nan2:PGO_NAN_HANDOFF=1" > $O/r05w_replay.txt 2>&1 || { tail -20 $O/r05w_replay.txt; exit 1; }
tail -1 $O/r05w_replay.txt
