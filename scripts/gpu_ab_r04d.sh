#!/bin/bash
# Round-4 A/B on the box: factorisation replays (1 / 3 lanes) and the live
# re-solve line under the round's switches (gather vs push assembly, split
# steps, far updates), then the per-level split of the default.
O=gpurun_out
bash scripts/gpu_ubench_wave_ab.sh > $O/r04d_ubench_wave.txt 2>&1 || { echo "ubench failed"; exit 1; }
grep -E "==|fronts|fingerprint" $O/r04d_ubench_wave.txt | paste - - | awk '{print $1, $2, $3, $4, $5, $6, $7, $8, $NF}'
timeout -k 10 600 python3 scripts/factor_breakdown.py --reps 10 --envs "default:PGO_DUMMY=1" "push:PGO_ASM_PUSH=1" \
  "nosplit:PGO_STEP_SPLIT=0" "far:PGO_FAR=1" "nowave2:PGO_WAVE2=0" "default2:PGO_DUMMY=2" > $O/r04d_ab.txt 2>&1 || { echo "ab failed"; exit 1; }
tail -6 $O/r04d_ab.txt
for v in default:PGO_DUMMY=1 push:PGO_ASM_PUSH=1 nosplit:PGO_STEP_SPLIT=0; do
  tag=${v%%:*}; kv=${v#*:}
  env $kv timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --marginals 0 --search 0 --gicp 0 \
    --gn 0 --live 6 > $O/r04d_live_$tag.json 2> $O/r04d_live_$tag.err || { echo "live $tag failed"; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/r04d_live_$tag.json').read().strip().splitlines()[-1]); l=d['live_resolve']; print('live $tag', round(l['ms_median'],1), [(round(x['ms'],1), round(x['ms_plan'],1), round(x['ms_upload'],1), x['lm_tries']) for x in l['per_registration']])"
done
bash scripts/gpu_levels.sh r04d > $O/r04d_levels.log 2>&1 || { echo "levels failed"; exit 1; }
grep -E "replay span|top level" $O/levels_r04d/levels_l*.txt
