#!/bin/bash
# Round 6 A/B: lambda lanes fused in one tile-assembly workgroup on levels of
# >= PGO_ASM_LANES_MIN tiles (default 2048; 0 = one workgroup per lane, as
# before): bitwise C2 / C3 and the single-GPU parity file, replays at 1 / 3
# lanes with thresholds 0 / 1024 / 2048 / 4096 (two rounds), short bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06aa
mkdir -p $O
for cfg in C2 C3; do
  for v in fused per_lane; do
    if [ $v = fused ]; then unset PGO_ASM_LANES_MIN; else export PGO_ASM_LANES_MIN=0; fi
    timeout -k 10 200 python3 scripts/bitwise_env_check.py --config $cfg --lanes 3 > $O/bitwise_${cfg}_$v.txt 2>&1 || { echo "bitwise $cfg $v failed"; tail -3 $O/bitwise_${cfg}_$v.txt; exit 1; }
    echo "$v $(tail -1 $O/bitwise_${cfg}_$v.txt)"
  done
done
unset PGO_ASM_LANES_MIN
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  timeout -k 10 600 python3 scripts/factor_breakdown.py --config C3 --lanes 1 2 3 \
    --envs "per_lane:PGO_ASM_LANES_MIN=0" "min1024:PGO_ASM_LANES_MIN=1024" "min4096:PGO_ASM_LANES_MIN=4096" > $O/replay$k.txt 2>&1 || exit 1
  tail -1 $O/replay$k.txt
done
for v in fused per_lane; do
  if [ $v = fused ]; then unset PGO_ASM_LANES_MIN; else export PGO_ASM_LANES_MIN=0; fi
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --c5 0 --live 0 --gicp 0 --marginals 0 --search 0 --gn 0 --converged 0 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || { echo "bench $v failed"; tail -5 $O/bench_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', 'it/s', round(d['value'],2), 'ms', round(d['ms_per_step'],2), 'fact', round(r['factorization']['frac'],4), 'err', d['per_step']['final_error'])"
done
unset PGO_ASM_LANES_MIN
echo done
