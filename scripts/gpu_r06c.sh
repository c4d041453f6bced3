#!/bin/bash
# Round 6: the diagonal tiles' factor + inverse by forward substitution
# (diag16_fs, the new default) against round 5's diag16_lane (build form 0,
# graphslam_amd/build/libpgo_form0.so): ubench, factorisation replays, the
# C3 / C5 parity tests that pin the trajectory, a short bench A/B.
O=gpurun_out
TAG=${TAG:-r06c}
L0=$PWD/graphslam_amd/build/libpgo_form0.so
timeout -k 10 60 ./graphslam_amd/build/ubench_factor64 > $O/${TAG}_ubench_factor64.txt 2>&1 || { echo "ubench failed"; exit 1; }
grep -E "total|per factor|PASS|FAIL" $O/${TAG}_ubench_factor64.txt
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  "tests/test_gpu_parity.py::test_cholesky_step_vs_oracle" "tests/test_gpu_parity.py::test_c3_full_size_against_golden" \
  tests/test_gpu_parity.py::test_c3_whole_trajectory_vs_numpy_twin tests/test_gpu_parity.py::test_c5_five_linearisations_against_fixture \
  tests/test_gpu_parity.py::test_c5_full_size_against_fixture -s > $O/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|rel diff|passed|failed|Error" $O/${TAG}_tests.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 scripts/factor_breakdown.py --config C3 --lanes 1 3 --envs "form0:PGO_LIB_PATH=$L0" > $O/${TAG}_replay.txt 2>&1 || exit 1
cat $O/${TAG}_replay.txt
for v in fs lane; do
  if [ $v = lane ]; then export PGO_LIB_PATH=$L0; else unset PGO_LIB_PATH; fi
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --c5 0 --live 0 --gicp 0 --marginals 0 --search 0 --gn 0 --converged 0 --no-cpu-baseline > $O/${TAG}_bench_$v.json 2> $O/${TAG}_bench_$v.err || { echo "bench $v failed"; tail -5 $O/${TAG}_bench_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/${TAG}_bench_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', 'it/s', round(d['value'],2), 'ms', round(d['ms_per_step'],2), 'k_step us', round(1e3*r['avg_launch_ms'],2), 'frac', round(r['frac'],4), 'fact', round(r['factorization']['frac'],4), 'err', d['per_step']['final_error'], 'retries', d['per_step']['handoff_retries'])"
done
echo done
