#!/bin/bash
# Round 5: fused look-ahead chain (the next diagonal factored by the workgroup
# that solves the column tile it reads).  GPU tests (parity, multi-rank bitwise
# vs one rank, determinism), bitwise A/B against PGO_FUSE_DIAG=0, the replay
# A/B, the bench.
O=gpurun_out
TAG=${TAG:-r05g}
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests -m gpu > $O/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
for cfg in C2 C3; do
  for v in 0 1; do
    PGO_FUSE_DIAG=$v timeout -k 10 200 python3 scripts/bitwise_env_check.py --config $cfg --lanes 3 > $O/${TAG}_fuse_${cfg}_$v.txt 2>&1 || exit 1
    echo "fuse=$v $(tail -1 $O/${TAG}_fuse_${cfg}_$v.txt)"
  done
done
timeout -k 10 400 python3 scripts/factor_breakdown.py --config C3 --lanes 1 3 --envs "nofuse:PGO_FUSE_DIAG=0" > $O/${TAG}_ab_fuse.txt 2>&1 || exit 1
tail -1 $O/${TAG}_ab_fuse.txt
timeout -k 10 700 python3 bench.py --c5 0 > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { echo "bench failed"; tail -5 $O/${TAG}_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/${TAG}_bench.json').read().strip().splitlines()[-1]); r=d['roofline']; print('bench', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'], r['factorization']['frac'], d['per_step']['final_error'])"
echo done
