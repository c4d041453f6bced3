#!/bin/bash
# Round 6 diagnostic: what bounds the tile assembly (k_assemble_tile)?
# Replays with the H-entry loads dropped (libpgo_nov.so, -DPGO_AB_NO_V) or the
# children's loads dropped (libpgo_noch.so, -DPGO_AB_NO_CH) -- wrong factors,
# times only -- against the product build; the assembly ablated; FETCH_SIZE /
# WRITE_SIZE of k_assemble_tile with and without the H-entry loads.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06v
mkdir -p $O
B=$PWD/graphslam_amd/build
timeout -k 10 500 python3 scripts/factor_breakdown.py --config C3 --lanes 1 3 \
  --envs "nov:PGO_LIB_PATH=$B/libpgo_nov.so" "noch:PGO_LIB_PATH=$B/libpgo_noch.so" > $O/replay.txt 2>&1 || exit 1
cat $O/replay.txt
timeout -k 10 300 python3 scripts/factor_breakdown.py --config C3 --lanes 1 3 --ablate assemble > $O/ablate.txt 2>&1 || exit 1
cat $O/ablate.txt
for v in prod nov; do
  if [ $v = prod ]; then unset PGO_LIB_PATH; else export PGO_LIB_PATH=$B/libpgo_$v.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c -T -f csv -d $O/pmc_${v}_$c -o c3 --kernel-include-regex "k_assemble_tile" -- \
      python3 bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-graphs --lanes 1 --max-outer 1 --live 0 --gicp 0 --search 0 --marginals 0 --c5 0 > $O/pmc_${v}_$c.log 2>&1
    rc=$?; echo "pmc $v $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
unset PGO_LIB_PATH
echo done
