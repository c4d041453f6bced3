#!/bin/bash
set -o pipefail
# A/B of two library builds (PGO_LIB_PATH); writes gpurun_out/ab.txt
mkdir -p gpurun_out
for lib in graphslam_amd/libpgo.so graphslam_amd/libpgo_b.so graphslam_amd/libpgo.so graphslam_amd/libpgo_b.so; do
  PGO_LIB_PATH=$PWD/$lib timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || exit $?
  grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', round(d['value'],3), d['linearize_kernel']['avg_launch_ms'])" | tee -a gpurun_out/ab.txt
done
