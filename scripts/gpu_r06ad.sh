#!/bin/bash
# Round 6 A/B: Schur-update deferral block kKB 512 / 128 against 256 (builds
# graphslam_amd/build/libpgo_kb512.so / _kb128.so): C3 trajectory (final error,
# tries) per build, replays at 1 / 3 lanes (two rounds), short bench each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ad
mkdir -p $O
B=$PWD/graphslam_amd/build
for v in kb256 kb512 kb128; do
  if [ $v = kb256 ]; then unset PGO_LIB_PATH; else export PGO_LIB_PATH=$B/libpgo_$v.so; fi
  timeout -k 10 200 python3 scripts/bitwise_env_check.py --config C3 --lanes 3 > $O/traj_$v.txt 2>&1 || { echo "traj $v failed"; tail -3 $O/traj_$v.txt; exit 1; }
  echo "$v $(tail -1 $O/traj_$v.txt)"
done
unset PGO_LIB_PATH
for k in 1 2; do
  timeout -k 10 500 python3 scripts/factor_breakdown.py --config C3 --lanes 1 3 \
    --envs "kb512:PGO_LIB_PATH=$B/libpgo_kb512.so" "kb128:PGO_LIB_PATH=$B/libpgo_kb128.so" > $O/replay$k.txt 2>&1 || exit 1
  tail -1 $O/replay$k.txt
done
for v in kb256 kb512; do
  if [ $v = kb256 ]; then unset PGO_LIB_PATH; else export PGO_LIB_PATH=$B/libpgo_$v.so; fi
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --c5 0 --live 0 --gicp 0 --marginals 0 --search 0 --gn 0 --converged 0 --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || { echo "bench $v failed"; tail -5 $O/bench_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; f=r['families']['k_panel_syrk_lds']; print('$v', 'it/s', round(d['value'],2), 'ms', round(d['ms_per_step'],2), 'fact', round(r['factorization']['frac'],4), 'syrk frac', round(f['frac'],4), 'err', d['per_step']['final_error'])"
done
unset PGO_LIB_PATH
echo done
