#!/bin/bash
# Small fronts, round 5: the trailing update's C loads one column block ahead and
# the inverse moved ahead of the trailing update (k_front_wave) -- old / new
# builds of scripts/ubench_wave.hip without phase stamps (launch time) and with
# (phases), on latency-bound (1-256 fronts) and throughput (4096-12288) launches;
# the output fingerprints must match old / new.  Then the replay times.
set -o pipefail
O=gpurun_out/r05t_wave.txt
: > $O
CFGS=("1 64 8" "256 64 8" "4096 64 8" "12288 64 8" "1 64 16" "256 64 16" "4096 64 16" "1 100 8" "256 100 8" "4096 100 8" "1 100 16" "256 100 16" "4096 100 16" "1 64 32" "256 64 32" "4096 64 32" "1 128 32")
for v in oldnc nc old new; do
  echo "== $v" >> $O
  for cfg in "${CFGS[@]}"; do timeout -k 5 60 ./graphslam_amd/build/ubench_wave_$v $cfg >> $O || exit 1; done
done
grep -E "^==|^fronts|fingerprint" $O | paste - - | head -80
timeout -k 10 300 python3 scripts/factor_breakdown.py --config C3 --lanes 1 3 > gpurun_out/r05t_replay.txt 2>&1 || exit 1
tail -2 gpurun_out/r05t_replay.txt
