#!/bin/bash
# A/B of the look-ahead front-height threshold (PGO_LOOKAHEAD_M) on the quick C3 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for m in ${LA_LIST:-2048 1024 512 4096}; do
  PGO_LOOKAHEAD_M=$m timeout -k 10 300 python3 bench.py --no-cpu-baseline --live 0 --gicp 0 --search 0 --marginals 0 \
    --profile-every 0 > gpurun_out/la_$m.log 2>&1 || { echo "m=$m failed"; tail -5 gpurun_out/la_$m.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/la_$m.log'):
    if l.startswith('{'):
        d = json.loads(l); print('M=$m value', round(d['value'], 3), 'fact ms', round(d['roofline']['factorization']['ms'] / d['roofline']['factorization']['factorizations'], 3))
"
done
