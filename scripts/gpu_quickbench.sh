#!/bin/bash
# Quick C3 bench (timed steps only, no CPU baseline or side benches) + root-level step stamps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --no-cpu-baseline --live 0 --gicp 0 --search 0 --marginals 0 ${BENCH_ARGS:-} \
  > gpurun_out/qb.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/qb.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/qb.log'):
    if l.startswith('{'):
        d = json.loads(l); print('value', round(d['value'], 3), 'ms/step', round(d['ms_per_step'], 1), 'fact ms', round(d['roofline']['factorization']['ms'] / d['roofline']['factorization']['factorizations'], 3))
"
[ "${STAMPS:-1}" = "1" ] && bash scripts/gpu_stamps.sh | tail -12
exit 0
