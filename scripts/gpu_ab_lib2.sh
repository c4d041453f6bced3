#!/bin/bash
# A/B of two library builds (PGO_LIB_PATH) on the default C3 bench without side lines
set -o pipefail
mkdir -p gpurun_out
for lib in graphslam_amd/libpgo.so graphslam_amd/libpgo_b.so graphslam_amd/libpgo.so graphslam_amd/libpgo_b.so; do
  PGO_LIB_PATH=$PWD/$lib timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --marginals 0 --search 0 --live 0 --gicp 0 > gpurun_out/ab.log 2>&1 || exit $?
  grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); f=d['roofline']['factorization']; print('$lib', round(d['value'],3), 'fact ms', round(f['ms']/f['factorizations'],3))"
done
