#!/bin/bash
# C5 (1M poses / 5M edges, 3 lambda lanes): one warm-up step (the plan's
# analysis), one timed step; no CPU baseline or side lines.
O=gpurun_out
TAG=${TAG:-r04c5}
timeout -k 10 900 python3 -u bench.py --config C5 --no-cpu-baseline --steps 1 --warmup 1 --marginals 0 --search 0 --gicp 0 \
  --gn 0 --converged 0 --live 0 > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { echo "c5 failed"; tail -5 $O/${TAG}_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/${TAG}_bench.json').read().strip().splitlines()[-1]); r=d['roofline']; f=r.get('factorization', {}); print('c5', d['value'], d['ms_per_step'], f.get('frac'), f.get('ms'), f.get('factorizations'))"
