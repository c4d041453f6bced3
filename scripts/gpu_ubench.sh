#!/bin/bash
# Microbenchmarks of Cholesky building blocks (built here, run on the GPU box).
set -o pipefail
mkdir -p gpurun_out
for cfg in "1 64" "64 64" "16 1024"; do
  timeout -k 10 120 ./graphslam_amd/build/ubench_diag $cfg || exit $?
done
