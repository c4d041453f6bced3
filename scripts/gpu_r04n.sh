#!/bin/bash
# Diagonal tiles factored over their live 16-column blocks only (default) vs
# all four (PGO_DIAG_FULL=1): bitwise check, replay A/B; GPU tests; bench line.
O=gpurun_out
TAG=${TAG:-r04n}
for v in 0 1; do
  PGO_DIAG_FULL=$v timeout -k 10 200 python3 scripts/bitwise_env_check.py --lanes 3 || { echo "check $v failed"; exit 1; }
done
timeout -k 10 400 python3 scripts/factor_breakdown.py --reps 10 --envs "full:PGO_DIAG_FULL=1" "default2:PGO_DUMMY=2" \
  "fullb:PGO_DIAG_FULL=1" > $O/${TAG}_ab.txt 2>&1 || { echo "ab failed"; tail -5 $O/${TAG}_ab.txt; exit 1; }
grep -v "^{" $O/${TAG}_ab.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { echo "bench failed"; exit 1; }
python3 -c "import json; d=json.loads(open('$O/${TAG}_bench.json').read().strip().splitlines()[-1]); l=d['live_resolve']; print('bench', round(d['value'],2), round(d['ms_per_step'],1), d['per_step']['final_error'], 'live', round(l['ms_median'],1), [round(x['ms'],1) for x in l['per_registration']])"
