#!/bin/bash
# Look-ahead threshold 512 as the default: GPU tests, then the headline under
# 2 / 3 / 4 lambda lanes (bench lines without the side lines).
O=gpurun_out
TAG=${TAG:-r04l}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
for L in 3 2 4 3; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 --lanes $L --marginals 0 --search 0 --gicp 0 --live 0 --gn 0 \
    --converged 0 > $O/${TAG}_bench_l$L.json 2> $O/${TAG}_bench_l$L.err || { echo "bench $L failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/${TAG}_bench_l$L.json').read().strip().splitlines()[-1]); print('lanes $L', round(d['value'],2), round(d['ms_per_step'],1), d['per_step']['final_error'])"
done
