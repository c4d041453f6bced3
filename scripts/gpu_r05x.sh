#!/bin/bash
# The frontal vectors in the tile assembly's launch (default; PGO_VEC_FUSE=0:
# their own launch on a side stream): bitwise C2 / C3 against the known
# results, replay A/B, then the GPU tests.
set -o pipefail
O=gpurun_out
: > $O/r05x_bitwise.txt
timeout -k 10 200 python3 scripts/bitwise_env_check.py --config C3 --lanes 3 >> $O/r05x_bitwise.txt 2>&1 || { tail -20 $O/r05x_bitwise.txt; exit 1; }
timeout -k 10 200 python3 scripts/bitwise_env_check.py --config C3 --lanes 1 >> $O/r05x_bitwise.txt 2>&1 || { tail -20 $O/r05x_bitwise.txt; exit 1; }
timeout -k 10 200 python3 scripts/bitwise_env_check.py --config C2 --lanes 1 >> $O/r05x_bitwise.txt 2>&1 || { tail -20 $O/r05x_bitwise.txt; exit 1; }
grep final $O/r05x_bitwise.txt
timeout -k 10 400 python3 scripts/factor_breakdown.py --config C3 --lanes 1 3 --envs "sep:PGO_VEC_FUSE=0" "fused:PGO_VEC_FUSE=1" "sep2:PGO_VEC_FUSE=0" > $O/r05x_replay.txt 2>&1 || { tail -20 $O/r05x_replay.txt; exit 1; }
tail -1 $O/r05x_replay.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r05x_tests.log 2>&1 || { tail -30 $O/r05x_tests.log; exit 1; }
tail -2 $O/r05x_tests.log
