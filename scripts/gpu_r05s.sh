#!/bin/bash
# Latency of the small-front kernels on the launch sizes the C3 schedule
# actually has (1 .. 300 fronts: most k_front_wave launches are latency-bound,
# r05y trace) -- the default build (W <= 16 one pivot at a time) against
# W = 16 in 8-column blocks (ubench_wave_pp8), and the two-wave kernel.
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/r05s_wave_latency.txt
: > $OUT
CFGS=("1 64 16" "16 64 16" "256 64 16" "1 100 16" "16 100 16" "256 100 16" "1 64 8" "256 64 8" "1 100 8" "1 64 32" "256 64 32" "1 128 32" "256 128 32" "4096 64 16")
for v in new pp8; do
  echo "== $v" >> $OUT
  for cfg in "${CFGS[@]}"; do timeout -k 5 60 ./graphslam_amd/build/ubench_wave_$v $cfg >> $OUT || exit 1; done
done
echo "== new, two waves (m > 64)" >> $OUT
for cfg in "1 100 16" "16 100 16" "256 100 16" "1 128 32" "256 128 32"; do UB_WAVE2=1 timeout -k 5 60 ./graphslam_amd/build/ubench_wave_new $cfg >> $OUT || exit 1; done
cat $OUT
# replay A/B: the small fronts' streams at the highest dispatch priority
timeout -k 10 400 python3 scripts/factor_breakdown.py --config C3 --lanes 1 3 --envs "prio:PGO_SMALL_PRIORITY=1" > gpurun_out/r05s_prio.txt 2>&1 || exit 1
tail -4 gpurun_out/r05s_prio.txt
