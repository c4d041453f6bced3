#!/bin/bash
# A/B of the one-wavefront small-front kernel (scripts/ubench_wave.hip) built
# from two trees (graphslam_amd/build/ubench_wave_old, _new): time per launch,
# per-phase clocks of front 0 and the bitwise output fingerprint.
for v in old new; do echo "== $v"; for cfg in "1 128 32" "4096 128 32" "4096 128 20" "4096 100 24" "4096 64 16" "4096 64 12" "4096 40 8" "4096 90 12"; do timeout -k 5 60 ./graphslam_amd/build/ubench_wave_$v $cfg || exit 1; done; done
