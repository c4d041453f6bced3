#!/bin/bash
# Round 6 A/B of a linearisation change against build/libpgo_prev.so: bitwise
# C2 / C3, then the bench line twice each way (linearize_kernel roofline).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r06z}
mkdir -p $O
B=$PWD/graphslam_amd/build
for cfg in C2 C3; do
  for v in new prev; do
    if [ $v = new ]; then unset PGO_LIB_PATH; else export PGO_LIB_PATH=$B/libpgo_prev.so; fi
    timeout -k 10 200 python3 scripts/bitwise_env_check.py --config $cfg --lanes 3 > $O/bitwise_${cfg}_$v.txt 2>&1 || { echo "bitwise $cfg $v failed"; tail -3 $O/bitwise_${cfg}_$v.txt; exit 1; }
    echo "$v $(tail -1 $O/bitwise_${cfg}_$v.txt)"
  done
done
for k in 1 2; do
  for v in new prev; do
    if [ $v = new ]; then unset PGO_LIB_PATH; else export PGO_LIB_PATH=$B/libpgo_prev.so; fi
    timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --c5 0 --live 0 --gicp 0 --marginals 0 --search 0 --gn 0 --converged 0 --no-cpu-baseline > $O/bench_${v}_$k.json 2> $O/bench_${v}_$k.err || { echo "bench $v failed"; tail -5 $O/bench_${v}_$k.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_${v}_$k.json').read().strip().splitlines()[-1]); r=d['roofline']; l=d['linearize_kernel']; print('$v', 'it/s', round(d['value'],2), 'ms', round(d['ms_per_step'],2), 'lin frac', round(l['frac'],4), {k: l[k] for k in l if 'ms' in k or 'us' in k})"
  done
done
unset PGO_LIB_PATH
echo done
