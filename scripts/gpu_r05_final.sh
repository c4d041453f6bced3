#!/bin/bash
# Round-5 evidence on the box (repo root): GPU tests, smoke, the default bench
# line (C3 headline + the C5 side line), then rocprofv3 kernel trace + stats
# and the FETCH_SIZE / WRITE_SIZE passes (scripts/gpu_profile.sh).
O=gpurun_out
TAG=${TAG:-r05z}
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests -m gpu > $O/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/${TAG}_smoke.log; exit 1; }
tail -3 $O/${TAG}_smoke.log
timeout -k 10 900 python3 bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { echo "bench failed"; tail -5 $O/${TAG}_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/${TAG}_bench.json').read().strip().splitlines()[-1]); r=d['roofline']; c5=d.get('c5') or {}; print('bench', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'], r['factorization']['frac'], d['cpu_baseline']['value'], 'c5', c5.get('value'))"
bash scripts/gpu_profile.sh || { echo "profile failed"; exit 1; }
echo done
