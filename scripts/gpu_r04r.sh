#!/bin/bash
# C5 (1M poses / 5M edges) bench line on the round-4 code, 3 lambda lanes.
O=gpurun_out
timeout -k 10 900 python3 bench.py --config C5 --steps 1 --warmup 0 --no-cpu-baseline --marginals 0 --search 0 --gicp 0 \
  --live 0 --gn 0 --converged 0 > $O/r04r_c5_bench.json 2> $O/r04r_c5_bench.err || { echo "c5 failed"; tail -5 $O/r04r_c5_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/r04r_c5_bench.json').read().strip().splitlines()[-1]); f=d['roofline']['factorization']; print('C5', round(d['value'],3), round(d['ms_per_step'],1), 'factor', round(f['achieved'],2), round(f['frac'],3), d['per_step']['lambda_rounds'], d['per_step']['solves_rank0'])"
