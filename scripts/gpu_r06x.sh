#!/bin/bash
# Round 6 A/B: elements per load group in the tile assembly (PGO_ASM_GE 16 / 4
# builds against the product's 8) and two children per group (PGO_ASM_UNROLL=2):
# replays (two rounds); bitwise C3 for each build.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06x
mkdir -p $O
B=$PWD/graphslam_amd/build
for v in ge16 ge4; do
  PGO_LIB_PATH=$B/libpgo_$v.so timeout -k 10 200 python3 scripts/bitwise_env_check.py --config C3 --lanes 3 > $O/bitwise_$v.txt 2>&1 || { echo "bitwise $v failed"; exit 1; }
  echo "$v $(tail -1 $O/bitwise_$v.txt)"
done
for k in 1 2; do
  timeout -k 10 500 python3 scripts/factor_breakdown.py --config C3 --lanes 1 3 \
    --envs "ge16:PGO_LIB_PATH=$B/libpgo_ge16.so" "ge4:PGO_LIB_PATH=$B/libpgo_ge4.so" "unroll2:PGO_ASM_UNROLL=2" > $O/replay$k.txt 2>&1 || exit 1
  tail -1 $O/replay$k.txt
done
echo done
