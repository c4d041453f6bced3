#!/bin/bash
# Round 5: replay A/B of the inline plain-tile threshold (k_step carries up to
# PGO_INLINE_TILES Schur tiles of a step instead of a concurrent launch on a side
# stream: no fork / join edges), bitwise check of the largest setting.
O=gpurun_out
timeout -k 10 500 python3 scripts/factor_breakdown.py --config C3 --lanes 1 3 --envs "i1024:PGO_INLINE_TILES=1024" "i2048:PGO_INLINE_TILES=2048" "i8192:PGO_INLINE_TILES=8192" > $O/r05q_inline.txt 2>&1 || exit 1
tail -1 $O/r05q_inline.txt
PGO_INLINE_TILES=8192 timeout -k 10 200 python3 scripts/bitwise_env_check.py --config C3 --lanes 3 > $O/r05q_bitwise.txt 2>&1 || exit 1
tail -1 $O/r05q_bitwise.txt
echo done
