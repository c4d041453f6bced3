#!/bin/bash
# Round 6 A/B against the previous commit's build (graphslam_amd/build/libpgo_prev.so):
# bitwise check (C2 / C3 final error + pose hash), replays, short bench each,
# and the poisoned-workspace / step-split / partition tests on the new build.
O=gpurun_out
TAG=${TAG:-r06g}
B=$PWD/graphslam_amd/build
for cfg in C2 C3; do
  for v in new prev; do
    if [ $v = new ]; then unset PGO_LIB_PATH; else export PGO_LIB_PATH=$B/libpgo_prev.so; fi
    timeout -k 10 200 python3 scripts/bitwise_env_check.py --config $cfg --lanes 3 > $O/${TAG}_bitwise_${cfg}_$v.txt 2>&1 || { echo "bitwise $cfg $v failed"; tail -3 $O/${TAG}_bitwise_${cfg}_$v.txt; exit 1; }
    echo "$v $(tail -1 $O/${TAG}_bitwise_${cfg}_$v.txt)"
  done
done
unset PGO_LIB_PATH
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py::test_poisoned_workspace_bitwise tests/test_gpu_parity.py::test_step_split_bitwise_fresh_processes \
  "tests/test_multi_gpu.py::test_partitioned_factorisation_matches_one_rank" tests/test_multi_gpu.py::test_partitioned_poisoned_workspace_bitwise \
  > $O/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 scripts/factor_breakdown.py --config C3 --lanes 1 3 --envs "prev:PGO_LIB_PATH=$B/libpgo_prev.so" > $O/${TAG}_replay.txt 2>&1 || exit 1
cat $O/${TAG}_replay.txt
for v in new prev; do
  if [ $v = new ]; then unset PGO_LIB_PATH; else export PGO_LIB_PATH=$B/libpgo_$v.so; fi
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --c5 0 --live 0 --gicp 0 --marginals 0 --search 0 --gn 0 --converged 0 --no-cpu-baseline > $O/${TAG}_bench_$v.json 2> $O/${TAG}_bench_$v.err || { echo "bench $v failed"; tail -5 $O/${TAG}_bench_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/${TAG}_bench_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', 'it/s', round(d['value'],2), 'ms', round(d['ms_per_step'],2), 'k_step us', round(1e3*r['avg_launch_ms'],2), 'frac', round(r['frac'],4), 'fact', round(r['factorization']['frac'],4), 'err', d['per_step']['final_error'], 'retries', d['per_step']['handoff_retries'])"
done
echo done
