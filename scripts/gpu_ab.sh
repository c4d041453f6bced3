#!/bin/bash
# A/B bench lines under environment settings given as arguments, e.g.
#   bash scripts/gpu_ab.sh "PGO_FUSE_FLOPS=0" "PGO_FUSE_FLOPS=4e8"
set -o pipefail
mkdir -p gpurun_out
for cfg in "$@"; do
  env $cfg timeout -k 10 ${T_BENCH:-240} python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab.log 2>&1
  rc=$?
  v=$(grep '^{' gpurun_out/ab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],3), round(d['ms_per_step'],1))")
  echo "$cfg -> rc=$rc $v" | tee -a gpurun_out/ab.txt
  [ $rc -eq 0 ] || exit $rc
done
