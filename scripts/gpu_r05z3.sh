#!/bin/bash
# The backward solve's chain with two blocks per workgroup (PGO_BWD_PAIR,
# default 1; 0: one block each): bitwise C2 / C3 results, the headline step
# A/B (bench.py, 3 timed steps each, alternating), then the GPU tests.
set -o pipefail
O=gpurun_out
: > $O/r05z3_bitwise.txt
for v in 1 0; do
  PGO_BWD_PAIR=$v timeout -k 10 200 python3 scripts/bitwise_env_check.py --config C3 --lanes 3 >> $O/r05z3_bitwise.txt 2>&1 || { tail -20 $O/r05z3_bitwise.txt; exit 1; }
  PGO_BWD_PAIR=$v timeout -k 10 200 python3 scripts/bitwise_env_check.py --config C2 --lanes 1 >> $O/r05z3_bitwise.txt 2>&1 || { tail -20 $O/r05z3_bitwise.txt; exit 1; }
done
grep final $O/r05z3_bitwise.txt
for v in 1 0 1 0; do
  PGO_BWD_PAIR=$v timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --live 0 --gicp 0 --search 0 --marginals 0 --c5 0 --gn 0 --converged 0 --profile-every 0 > $O/r05z3_b$v.json 2> $O/r05z3_b$v.err || { echo "bench $v failed"; tail -3 $O/r05z3_b$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/r05z3_b$v.json').read().strip().splitlines()[-1]); print('PGO_BWD_PAIR=$v', round(d['value'],2), round(d['ms_per_step'],2), d['per_step']['final_error'])" | tee -a $O/r05z3_bench.txt
done
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r05z3_tests.log 2>&1 || { tail -30 $O/r05z3_tests.log; exit 1; }
tail -2 $O/r05z3_tests.log
