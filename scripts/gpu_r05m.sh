#!/bin/bash
# Round 5: the diagonal tiles' L no longer stored (dead stores) and the tile
# assembly's index loads in three rounds: the factor
# microbenchmark, GPU tests, bitwise check against the previous build's C2 / C3
# results, replay time, bench.
O=gpurun_out
TAG=${TAG:-r05m}
timeout -k 10 60 ./graphslam_amd/build/ubench_factor64 > $O/${TAG}_ubench_factor64.txt 2>&1 || { echo "ubench failed"; cat $O/${TAG}_ubench_factor64.txt; exit 1; }
cat $O/${TAG}_ubench_factor64.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests -m gpu > $O/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
for cfg in C2 C3; do
  timeout -k 10 200 python3 scripts/bitwise_env_check.py --config $cfg --lanes 3 > $O/${TAG}_bitwise_${cfg}.txt 2>&1 || exit 1
  tail -1 $O/${TAG}_bitwise_${cfg}.txt
done
timeout -k 10 400 python3 scripts/factor_breakdown.py --config C3 --lanes 1 3 --envs > $O/${TAG}_replay.txt 2>&1 || exit 1
tail -1 $O/${TAG}_replay.txt
timeout -k 10 700 python3 bench.py --c5 0 > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { echo "bench failed"; tail -5 $O/${TAG}_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/${TAG}_bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print('bench', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'], r['factorization']['frac'], d['per_step']['final_error'])"
echo done
