#!/bin/bash
# Round-6 evidence on the box (repo root): the default bench line (C3 headline
# + the C5 side line + the CPU baseline), then rocprofv3 kernel trace + stats
# and the FETCH_SIZE / WRITE_SIZE passes (scripts/gpu_profile.sh).  The GPU
# suite and smoke run in their own call (scripts/gpu_r06d.sh).
O=gpurun_out
TAG=${TAG:-r06f}
timeout -k 10 900 python3 bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { echo "bench failed"; tail -5 $O/${TAG}_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/${TAG}_bench.json').read().strip().splitlines()[-1]); r=d['roofline']; c5=d.get('c5') or {}; print('bench', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'], r['factorization']['frac'], d['cpu_baseline']['value'], d['cpu_baseline']['gpu_over_cpu'], d['cpu_baseline']['gpu_over_cpu_one_core'], 'c5', c5.get('value'), 'retries', d['per_step']['handoff_retries'])"
bash scripts/gpu_profile.sh || { echo "profile failed"; exit 1; }
echo done
