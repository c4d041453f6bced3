#!/bin/bash
# Round 6 A/B: the Cholesky-mode V as one 72-byte record per factor (V[9 e + q])
# instead of nine arrays, against the previous commit (build/libpgo_prev.so):
# bitwise C2 / C3, the single-GPU parity file, replays, FETCH / WRITE of the
# assembly and the linearisation, short bench each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06y
mkdir -p $O
B=$PWD/graphslam_amd/build
for cfg in C2 C3; do
  for v in new prev; do
    if [ $v = new ]; then unset PGO_LIB_PATH; else export PGO_LIB_PATH=$B/libpgo_prev.so; fi
    timeout -k 10 200 python3 scripts/bitwise_env_check.py --config $cfg --lanes 3 > $O/bitwise_${cfg}_$v.txt 2>&1 || { echo "bitwise $cfg $v failed"; tail -3 $O/bitwise_${cfg}_$v.txt; exit 1; }
    echo "$v $(tail -1 $O/bitwise_${cfg}_$v.txt)"
  done
done
unset PGO_LIB_PATH
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 scripts/factor_breakdown.py --config C3 --lanes 1 3 --envs "prev:PGO_LIB_PATH=$B/libpgo_prev.so" > $O/replay.txt 2>&1 || exit 1
tail -1 $O/replay.txt
for v in new prev; do
  if [ $v = new ]; then unset PGO_LIB_PATH; else export PGO_LIB_PATH=$B/libpgo_prev.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c -T -f csv -d $O/pmc_${v}_$c -o c3 --kernel-include-regex "k_assemble_tile|k_linearize" -- \
      python3 bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-graphs --lanes 1 --max-outer 1 --live 0 --gicp 0 --search 0 --marginals 0 --c5 0 > $O/pmc_${v}_$c.log 2>&1
    rc=$?; echo "pmc $v $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
for v in new prev; do
  if [ $v = new ]; then unset PGO_LIB_PATH; else export PGO_LIB_PATH=$B/libpgo_prev.so; fi
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --c5 0 --live 0 --gicp 0 --marginals 0 --search 0 --gn 0 --converged 0 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || { echo "bench $v failed"; tail -5 $O/bench_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', 'it/s', round(d['value'],2), 'ms', round(d['ms_per_step'],2), 'fact', round(r['factorization']['frac'],4), 'lin', round(d['linearize_kernel']['frac'],4) if d.get('linearize_kernel') else None, 'err', d['per_step']['final_error'])"
done
unset PGO_LIB_PATH
echo done
