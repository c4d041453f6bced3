#!/bin/bash
# Round-4 check on the box (repo root): GPU tests, the small-front
# microbenchmark A/B, factorisation replay A/B of the two-wave choice, the
# default bench line and the live re-solve line.
O=gpurun_out
TAG=${TAG:-r04f}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ubench_wave_ab.sh > $O/${TAG}_ubench_wave.txt 2>&1 || { echo "ubench failed"; exit 1; }
grep -E "^==|^fronts" $O/${TAG}_ubench_wave.txt
timeout -k 10 400 python3 scripts/factor_breakdown.py --reps 10 --envs "default:PGO_DUMMY=1" "nowave2:PGO_WAVE2=0" \
  "wave2all:PGO_WAVE2=2" "default2:PGO_DUMMY=2" > $O/${TAG}_ab.txt 2>&1 || { echo "ab failed"; exit 1; }
tail -1 $O/${TAG}_ab.txt
timeout -k 10 400 python3 bench.py --steps 5 > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { echo "bench failed"; exit 1; }
python3 -c "import json; d=json.loads(open('$O/${TAG}_bench.json').read().strip().splitlines()[-1]); l=d['live_resolve']; print('bench', d['value'], d['ms_per_step'], 'live', round(l['ms_median'],1), [(round(x['ms'],1), round(x['ms_plan'],1), round(x['ms_upload'],1), round(x['ms_optimize'],1)) for x in l['per_registration']])"
echo done
