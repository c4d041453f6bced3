#!/bin/bash
# C5 bench with and without the look-ahead skip (one step each)
set -o pipefail
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --config C5 --steps 1 --warmup 0 --no-cpu-baseline --marginals 0 --search 0 --live 0 --gicp 0 > gpurun_out/ab5_$tag.log 2>&1
  local rc=$?; [ $rc -eq 0 ] || { echo "$tag rc=$rc"; exit $rc; }
  grep '^{' gpurun_out/ab5_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); f=d['roofline']['factorization']; print('$tag', round(d['value'],3), round(d['ms_per_step'],1), 'fact ms', round(f['ms']/f['factorizations'],3), 'frac', round(f['frac'],4))"
}
run look X=1
run nolook PGO_NO_LOOKAHEAD=1
