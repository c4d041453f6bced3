#!/bin/bash
# A/B of environment switches on the default C3 bench (no side lines): one line per setting
set -o pipefail
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --marginals 0 --search 0 --live 0 --gicp 0 > gpurun_out/ab_$tag.log 2>&1
  local rc=$?; [ $rc -eq 0 ] || { echo "$tag rc=$rc"; exit $rc; }
  grep '^{' gpurun_out/ab_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); f=d['roofline']['factorization']; print('$tag', round(d['value'],3), round(d['ms_per_step'],1), 'fact ms', round(f['ms']/f['factorizations'],3))"
}
run base X=1
run nolook PGO_NO_LOOKAHEAD=1
run noprio PGO_SIDE_PRIORITY=0
run nolook_noprio PGO_NO_LOOKAHEAD=1 PGO_SIDE_PRIORITY=0
