# A/B of the lambda-lane sizing rule (PGO_LANES_ADAPT 1: LM-dynamics rule, 2: previous count)
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for A in 1 3; do
    PGO_LANES_ADAPT=$A timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 5 --marginals 0 --search 0 --gicp 0 --live 0 --gn 0 --converged 0 > gpurun_out/ab/c3_a$A.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/ab/c3_a$A.json').read().strip().splitlines()[-1]); print('C3 adapt $A', round(d['value'],2), round(d['ms_per_step'],1), d['per_step']['lambda_rounds'], d['per_step']['solves_rank0'], d['per_step']['final_error'])"
  done
done
for A in 1 3; do
  PGO_LANES_ADAPT=$A timeout -k 10 300 python3 bench.py --config C5 --no-cpu-baseline --steps 1 --warmup 1 --marginals 0 --search 0 --gicp 0 --live 0 --gn 0 --converged 0 > gpurun_out/ab/c5_a$A.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ab/c5_a$A.json').read().strip().splitlines()[-1]); print('C5 adapt $A', round(d['value'],3), round(d['ms_per_step'],1), d['per_step']['lambda_rounds'], d['per_step']['solves_rank0'], d['per_step']['final_error'])"
done
