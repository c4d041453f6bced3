#!/bin/bash
# Round-4 final evidence on the box (repo root): GPU tests, smoke, the default
# bench line, then rocprofv3 kernel trace + stats and the FETCH_SIZE /
# WRITE_SIZE passes (scripts/gpu_profile.sh).
O=gpurun_out
TAG=${TAG:-r04z}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/${TAG}_smoke.log; exit 1; }
tail -3 $O/${TAG}_smoke.log
timeout -k 10 400 python3 bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { echo "bench failed"; tail -5 $O/${TAG}_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/${TAG}_bench.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['cpu_baseline']['value'])"
bash scripts/gpu_profile.sh || { echo "profile failed"; exit 1; }
echo done
