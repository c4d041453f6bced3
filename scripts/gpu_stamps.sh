#!/bin/bash
# In-kernel wall-clock stamps of the root level's panel steps (PGO_STEP_STAMPS):
# per step, stamps 1..4 of the diagonal workgroup (update, factor+inverse,
# publish, store) and 5..8 of the first waiting workgroup, in us from its start.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/stamps_${TAG:-q}
mkdir -p $OUT && rm -f $OUT/dump.txt
PGO_STEP_STAMPS=1 PGO_PROFILE_DUMP=$OUT/dump.txt timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 \
  --no-cpu-baseline --live 0 --gicp 0 --search 0 --marginals 0 ${BENCH_ARGS:-} > $OUT/bench.log 2>&1
rc=$?; echo "rc=$rc"; grep "# stamp" $OUT/dump.txt | tail -70
exit $rc
