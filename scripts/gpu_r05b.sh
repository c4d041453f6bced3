#!/bin/bash
# Round 5: the new determinism tests (NaN-poisoned workspace, split steps in
# fresh processes), the hybrid multi-GPU tests (ranks sharing the GPU), the
# default bench line with the C5 side line, replay times per lane count.
O=gpurun_out
TAG=${TAG:-r05b}
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_multi_gpu.py -m gpu \
  -k "poison or split_bitwise or save_restore or rezeroed or (hybrid and not C5)" > $O/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python3 bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { echo "bench failed"; tail -5 $O/${TAG}_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/${TAG}_bench.json').read().strip().splitlines()[-1]); c=d['c5']; print('bench', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['cpu_baseline']['value'], d['per_step']['tries_per_linearization']); print('c5', c['value'], c['ms_per_optimize'], c['factorization'], c['lm_tries'], c['lambda_rounds'], c['tries_per_linearization'])"
timeout -k 10 300 python3 scripts/factor_breakdown.py --config C3 --lanes 1 2 3 --envs > $O/${TAG}_lanes_C3.txt 2>&1 || exit 1
tail -1 $O/${TAG}_lanes_C3.txt
echo done
