#!/bin/bash
# Graph-mode factorisation time with launch families removed (PGO_ABLATE,
# diagnostics: the factor is wrong in every run but the first)
set -o pipefail
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --marginals 0 --search 0 --live 0 --gicp 0 > gpurun_out/abl_$tag.log 2>&1
  local rc=$?; [ $rc -eq 0 ] || { echo "$tag rc=$rc"; tail -3 gpurun_out/abl_$tag.log; return 0; }
  grep '^{' gpurun_out/abl_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); f=d['roofline']['factorization']; print('$tag', 'fact ms', round(f['ms']/f['factorizations'],3), 'n', f['factorizations'])"
}
run none X=1
for a in small plain assemble vec first step small,plain step,plain; do run $a PGO_ABLATE=$a; done
