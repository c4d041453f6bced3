#!/bin/bash
# A/B of the small-front kernels (scripts/ubench_wave.hip): the default build
# (graphslam_amd/build/ubench_wave_new: W <= 16 one pivot at a time, W = 32 in
# 8-column blocks), a build with every class one pivot at a time
# (ubench_wave_pp32, -DPGO_WAVE_PERPIVOT_W=32) and, for m > 64, the two-wave
# kernel (UB_WAVE2=1): time per launch, per-phase clocks of front 0 and the
# bitwise output fingerprint (equal fingerprints: bitwise the same fronts).
CFGS=("1 128 32" "4096 128 32" "4096 100 24" "4096 90 12" "4096 64 16" "4096 64 24" "4096 56 32" "4096 48 20" "4096 40 8")
for v in new pp32; do echo "== $v"; for cfg in "${CFGS[@]}"; do timeout -k 5 60 ./graphslam_amd/build/ubench_wave_$v $cfg || exit 1; done; done
echo "== new, two waves (m > 64)"; for cfg in "${CFGS[@]}"; do UB_WAVE2=1 timeout -k 5 60 ./graphslam_amd/build/ubench_wave_new $cfg || exit 1; done
