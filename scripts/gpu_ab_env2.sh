#!/bin/bash
# A/B of the look-ahead threshold / apart policy on the default C3 bench (no side lines)
set -o pipefail
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --marginals 0 --search 0 --live 0 --gicp 0 > gpurun_out/ab_$tag.log 2>&1
  local rc=$?; [ $rc -eq 0 ] || { echo "$tag rc=$rc"; tail -3 gpurun_out/ab_$tag.log; exit $rc; }
  grep '^{' gpurun_out/ab_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); f=d['roofline']['factorization']; print('$tag', round(d['value'],3), round(d['ms_per_step'],1), 'fact ms', round(f['ms']/f['factorizations'],3), 'tries', d['per_step']['lm_tries'])"
}
run base X=1
run m512 PGO_LOOKAHEAD_M=512
run m512_apart PGO_LOOKAHEAD_M=512 PGO_APART_SKIP=1
run m256_apart PGO_LOOKAHEAD_M=256 PGO_APART_SKIP=1
run m2048_apart PGO_APART_SKIP=1
