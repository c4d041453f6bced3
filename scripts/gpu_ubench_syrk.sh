#!/bin/bash
set -o pipefail
for cfg in "1024 512" "2048 512" "4096 512"; do
  timeout -k 10 120 ./graphslam_amd/build/ubench_syrk $cfg || exit $?
done
