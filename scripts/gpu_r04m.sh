#!/bin/bash
# Four-wave small fronts (128 < m <= 256, w <= 32; PGO_WAVE4=0: the blocked
# path as before): GPU tests, replay A/B, bench line.
O=gpurun_out
TAG=${TAG:-r04m}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/${TAG}_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/${TAG}_tests.log | head -20; exit $rc; }
timeout -k 10 400 python3 scripts/factor_breakdown.py --reps 10 --envs "nowave4:PGO_WAVE4=0" "default2:PGO_DUMMY=2" \
  "nowave4b:PGO_WAVE4=0" > $O/${TAG}_ab.txt 2>&1 || { echo "ab failed"; tail -5 $O/${TAG}_ab.txt; exit 1; }
grep -v "^{" $O/${TAG}_ab.txt
for v in 1 0; do
  PGO_WAVE4=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --marginals 0 --search 0 --gicp 0 --live 0 --gn 0 \
    --converged 0 > $O/${TAG}_bench_w$v.json 2> $O/${TAG}_bench_w$v.err || { echo "bench $v failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/${TAG}_bench_w$v.json').read().strip().splitlines()[-1]); print('wave4 $v', round(d['value'],2), round(d['ms_per_step'],1), d['per_step']['final_error'])"
done
