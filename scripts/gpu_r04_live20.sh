#!/bin/bash
# The live line over 20 registrations (plan update and registration times), C3,
# from the optimum as in the default bench (the converged-regime line first).
O=gpurun_out
TAG=${TAG:-r04l20}
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 1 --warmup 0 --marginals 0 --search 0 --gicp 0 \
  --gn 0 --live 20 > $O/${TAG}_live.json 2> $O/${TAG}_live.err || { echo "live failed"; tail -5 $O/${TAG}_live.err; exit 1; }
python3 -c "
import json, statistics as st
d = json.loads(open('$O/${TAG}_live.json').read().strip().splitlines()[-1]); l = d['live_resolve']['per_registration']
ms = [x['ms'] for x in l]; pl = [x['ms_plan'] for x in l]
print('live n', len(l), 'ms median %.1f max %.1f' % (st.median(ms), max(ms)), 'plan median %.2f max %.2f' % (st.median(pl), max(pl)))"
