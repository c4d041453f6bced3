#!/bin/bash
# Round-4 GPU check (run on the box from the repo root): the small-front
# microbenchmark A/B, a default bench line, the far-update A/B, the live
# re-solve phase timings, then the GPU test suite.  TAG names the outputs.
TAG=${TAG:-r04c}
O=gpurun_out
bash scripts/gpu_ubench_wave_ab.sh > $O/${TAG}_ubench_wave.txt 2>&1; echo "ubench rc=$?"
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 5 > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { echo "bench failed"; exit 1; }
echo "bench ok"
timeout -k 10 400 python3 scripts/factor_breakdown.py --reps 10 --envs "far:PGO_DUMMY=1" "nofar:PGO_NO_FAR=1" \
  "far_defprio:PGO_FAR_PRIORITY=0" "nosplit:PGO_STEP_SPLIT=0" > $O/${TAG}_ab_far.txt 2>&1 || { echo "ab failed"; exit 1; }
echo "ab ok"
PGO_PLAN_TIMING=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --marginals 0 --search 0 \
  --gicp 0 --gn 0 --converged 0 --live 3 > $O/${TAG}_live.json 2> $O/${TAG}_live_timing.log || { echo "live failed"; exit 1; }
echo "live ok"
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests -m gpu > $O/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/${TAG}_tests.log
exit $rc
