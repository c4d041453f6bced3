#!/bin/bash
# Recheck of the committed small-front form (m <= 64 branch: the previous
# source verbatim; m > 64: one block ahead): old / new ubench fingerprints and
# launch times, replay times, bitwise C3 across two fresh processes.
set -o pipefail
O=gpurun_out/r05v_wave.txt
: > $O
CFGS=("1 64 8" "12288 64 8" "1 64 16" "1 100 8" "256 100 8" "2400 100 8" "1 100 16" "256 100 16" "4096 100 16")
W2=("1 128 32" "256 128 32" "5400 128 32")
for v in oldnc nc; do
  echo "== $v" >> $O
  for cfg in "${CFGS[@]}"; do timeout -k 5 60 ./graphslam_amd/build/ubench_wave_$v $cfg >> $O || exit 1; done
  echo "== $v two waves" >> $O
  for cfg in "${W2[@]}"; do UB_WAVE2=1 timeout -k 5 60 ./graphslam_amd/build/ubench_wave_$v $cfg >> $O || exit 1; done
done
grep -E "^==|^fronts|fingerprint" $O | paste - - | head -80
timeout -k 10 300 python3 scripts/factor_breakdown.py --config C3 --lanes 1 3 > gpurun_out/r05v_replay.txt 2>&1 || exit 1
tail -1 gpurun_out/r05v_replay.txt
timeout -k 10 200 python3 scripts/bitwise_env_check.py --config C3 --lanes 3 > gpurun_out/r05v_bitwise.txt 2>&1 || exit 1
tail -2 gpurun_out/r05v_bitwise.txt
