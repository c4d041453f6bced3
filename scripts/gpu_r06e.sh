#!/bin/bash
# Round 6 A/B: trsm_rows' inverse fragments straight from memory (default)
# against the LDS-staged form (graphslam_amd/build/libpgo_trsm0.so): replays,
# a short bench each, and the trajectory tests (bitwise: same products).
O=gpurun_out
TAG=${TAG:-r06e}
B=$PWD/graphslam_amd/build
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py::test_c3_full_size_against_golden tests/test_gpu_parity.py::test_poisoned_workspace_bitwise \
  tests/test_gpu_parity.py::test_lm_parity_with_golden > $O/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 scripts/factor_breakdown.py --config C3 --lanes 1 3 --envs "trsm0:PGO_LIB_PATH=$B/libpgo_trsm0.so" > $O/${TAG}_replay.txt 2>&1 || exit 1
cat $O/${TAG}_replay.txt
for v in new trsm0; do
  if [ $v = new ]; then unset PGO_LIB_PATH; else export PGO_LIB_PATH=$B/libpgo_$v.so; fi
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --c5 0 --live 0 --gicp 0 --marginals 0 --search 0 --gn 0 --converged 0 --no-cpu-baseline > $O/${TAG}_bench_$v.json 2> $O/${TAG}_bench_$v.err || { echo "bench $v failed"; tail -5 $O/${TAG}_bench_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/${TAG}_bench_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', 'it/s', round(d['value'],2), 'ms', round(d['ms_per_step'],2), 'k_step us', round(1e3*r['avg_launch_ms'],2), 'frac', round(r['frac'],4), 'fact', round(r['factorization']['frac'],4), 'err', d['per_step']['final_error'], 'retries', d['per_step']['handoff_retries'])"
done
echo done
