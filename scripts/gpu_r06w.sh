#!/bin/bash
# Round 6 A/B: XCD-aware order of the tile-assembly tasks (ea_xcd_order) against
# the natural order (PGO_ASM_XCD=0): bitwise C2 / C3, plan / append / poison
# tests, replays (two rounds), k_assemble_tile FETCH_SIZE both ways, short bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06w
mkdir -p $O
for cfg in C2 C3; do
  for v in xcd natural; do
    if [ $v = xcd ]; then unset PGO_ASM_XCD; else export PGO_ASM_XCD=0; fi
    timeout -k 10 200 python3 scripts/bitwise_env_check.py --config $cfg --lanes 3 > $O/bitwise_${cfg}_$v.txt 2>&1 || { echo "bitwise $cfg $v failed"; tail -3 $O/bitwise_${cfg}_$v.txt; exit 1; }
    echo "$v $(tail -1 $O/bitwise_${cfg}_$v.txt)"
  done
done
unset PGO_ASM_XCD
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py::test_poisoned_workspace_bitwise tests/test_gpu_parity.py::test_incremental_append_matches_oracle \
  tests/test_gpu_parity.py::test_append_in_place_matches_full_upload tests/test_gpu_parity.py::test_registrations_plan_append_matches_oracle \
  tests/test_gpu_parity.py::test_incremental_loop_closure_inside_fill_keeps_plan tests/test_multi_gpu.py::test_partitioned_poisoned_workspace_bitwise \
  > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  timeout -k 10 400 python3 scripts/factor_breakdown.py --config C3 --lanes 1 3 --envs "natural:PGO_ASM_XCD=0" > $O/replay$k.txt 2>&1 || exit 1
  tail -1 $O/replay$k.txt
done
for v in xcd natural; do
  if [ $v = xcd ]; then unset PGO_ASM_XCD; else export PGO_ASM_XCD=0; fi
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -T -f csv -d $O/pmc_$v -o c3 --kernel-include-regex "k_assemble_tile" -- \
    python3 bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-graphs --lanes 1 --max-outer 1 --live 0 --gicp 0 --search 0 --marginals 0 --c5 0 > $O/pmc_$v.log 2>&1
  rc=$?; echo "pmc $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for v in xcd natural; do
  if [ $v = xcd ]; then unset PGO_ASM_XCD; else export PGO_ASM_XCD=0; fi
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --c5 0 --live 0 --gicp 0 --marginals 0 --search 0 --gn 0 --converged 0 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || { echo "bench $v failed"; tail -5 $O/bench_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', 'it/s', round(d['value'],2), 'ms', round(d['ms_per_step'],2), 'fact', round(r['factorization']['frac'],4), 'err', d['per_step']['final_error'])"
done
unset PGO_ASM_XCD
echo done
