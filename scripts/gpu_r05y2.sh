#!/bin/bash
# The W = 8 and W = 16 one-wave small-front classes in one launch per row class (default; PGO_WAVE_PAIR=0:
# two launches in a row): bitwise C2 / C3 against the known
# results, replay A/B, then the GPU tests.
set -o pipefail
O=gpurun_out
: > $O/r05y2_bitwise.txt
timeout -k 10 200 python3 scripts/bitwise_env_check.py --config C3 --lanes 3 >> $O/r05y2_bitwise.txt 2>&1 || { tail -20 $O/r05y2_bitwise.txt; exit 1; }
timeout -k 10 200 python3 scripts/bitwise_env_check.py --config C3 --lanes 1 >> $O/r05y2_bitwise.txt 2>&1 || { tail -20 $O/r05y2_bitwise.txt; exit 1; }
timeout -k 10 200 python3 scripts/bitwise_env_check.py --config C2 --lanes 1 >> $O/r05y2_bitwise.txt 2>&1 || { tail -20 $O/r05y2_bitwise.txt; exit 1; }
grep final $O/r05y2_bitwise.txt
timeout -k 10 400 python3 scripts/factor_breakdown.py --config C3 --lanes 1 3 --envs "sep:PGO_WAVE_PAIR=0" "pair:PGO_WAVE_PAIR=1" "sep2:PGO_WAVE_PAIR=0" "pair2:PGO_WAVE_PAIR=1" > $O/r05y2_replay.txt 2>&1 || { tail -20 $O/r05y2_replay.txt; exit 1; }
tail -1 $O/r05y2_replay.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r05y2_tests.log 2>&1 || { tail -30 $O/r05y2_tests.log; exit 1; }
tail -2 $O/r05y2_tests.log
