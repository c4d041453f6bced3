#!/bin/bash
# GPU tests on the bound-slot-code appends, then the live line with plan timings and a bench line.
O=gpurun_out
TAG=${TAG:-r04v}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/${TAG}_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/${TAG}_tests.log | head; exit $rc; }
PGO_PLAN_TIMING=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --marginals 0 --search 0 --gicp 0 \
  --gn 0 --live 5 > $O/${TAG}_live.json 2> $O/${TAG}_live_timing.log || { echo "live failed"; exit 1; }
python3 -c "import json; d=json.loads(open('$O/${TAG}_live.json').read().strip().splitlines()[-1]); l=d['live_resolve']; print('live', round(l['ms_median'],1), [(round(x['ms'],1), round(x['ms_plan'],1), round(x['ms_upload'],1)) for x in l['per_registration']])"
grep -E "ensure_chol|bind_plan" $O/${TAG}_live_timing.log | tail -8
