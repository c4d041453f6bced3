#!/bin/bash
# Round-4 validation + A/B on the box (repo root): the GPU test suite, the
# small-front microbenchmark (one vs two waves, bitwise fingerprints), the
# factorisation replay A/B over the round's switches, the live re-solve
# line (default and push assembly), from the optimum.
O=gpurun_out
TAG=${TAG:-r04e}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ubench_wave_ab.sh > $O/${TAG}_ubench_wave.txt 2>&1 || { echo "ubench failed"; exit 1; }
grep -E "==|fingerprint" $O/${TAG}_ubench_wave.txt | tail -24
timeout -k 10 400 python3 scripts/factor_breakdown.py --reps 10 --envs "default:PGO_DUMMY=1" "push:PGO_ASM_PUSH=1" \
  "nosplit:PGO_STEP_SPLIT=0" "nowave2:PGO_WAVE2=0" "default2:PGO_DUMMY=2" > $O/${TAG}_ab.txt 2>&1 || { echo "ab failed"; exit 1; }
tail -8 $O/${TAG}_ab.txt
for v in default:PGO_DUMMY=1 push:PGO_ASM_PUSH=1; do
  tag=${v%%:*}; kv=${v#*:}
  env $kv timeout -k 10 240 python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --marginals 0 --search 0 --gicp 0 \
    --gn 0 --live 6 > $O/${TAG}_live_$tag.json 2> $O/${TAG}_live_$tag.err || { echo "live $tag failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/${TAG}_live_$tag.json').read().strip().splitlines()[-1]); l=d['live_resolve']; print('live $tag', round(l['ms_median'],1), [(round(x['ms'],1), round(x['ms_plan'],1), round(x['ms_upload'],1), round(x['ms_optimize'],1), x['lm_tries']) for x in l['per_registration']])"
done
PGO_PLAN_TIMING=1 timeout -k 10 240 python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --marginals 0 --search 0 \
  --gicp 0 --gn 0 --live 3 > $O/${TAG}_live_timing.json 2> $O/${TAG}_live_timing.log || { echo "live timing failed"; exit 1; }
echo done
