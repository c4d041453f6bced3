#!/bin/bash
# Schur-update tile kernel A/B (scripts/ubench_syrk.hip): the LDS-staged 64x64
# kernel with the C tile loaded after the k loop (tile 65) or before it (66),
# on the outer update of a big front and of mid-level fronts.
for cfg in "4096 512" "2048 256" "1024 256" "640 128"; do
  timeout -k 5 120 ./graphslam_amd/build/ubench_syrk $cfg || exit 1
done
