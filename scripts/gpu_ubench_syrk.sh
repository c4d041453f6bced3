#!/bin/bash
set -o pipefail
for cfg in "2048 512" "4096 512"; do
  timeout -k 10 120 ./graphslam_amd/build/ubench_syrk $cfg || exit $?
  XCD=1 timeout -k 10 120 ./graphslam_amd/build/ubench_syrk $cfg || exit $?
done
