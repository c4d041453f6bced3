#!/bin/bash
# Round-5 baseline on the box: GPU tests, the default bench line, then the
# split-step knob: bitwise (final error + pose hash, fresh processes) and the
# replay A/B (scripts/factor_breakdown.py).
O=gpurun_out
TAG=${TAG:-r05a}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { echo "bench failed"; tail -5 $O/${TAG}_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/${TAG}_bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['cpu_baseline']['value'])"
for cfg in C2 C3; do
  for v in 0 64 1; do
    PGO_STEP_SPLIT=$v timeout -k 10 200 python3 scripts/bitwise_env_check.py --config $cfg --lanes 3 > $O/${TAG}_split_${cfg}_$v.txt 2>&1 || exit 1
    echo "split=$v $(cat $O/${TAG}_split_${cfg}_$v.txt | tail -1)"
  done
done
timeout -k 10 400 python3 scripts/factor_breakdown.py --lanes 1 3 --envs "nosplit:PGO_STEP_SPLIT=0" > $O/${TAG}_ab_split.txt 2>&1 || exit 1
cat $O/${TAG}_ab_split.txt | tail -6
echo done
