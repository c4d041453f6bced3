mkdir -p gpurun_out/lanes
for L in 2 3 4; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --lanes $L --steps 5 --marginals 0 --search 0 --gicp 0 --live 0 --gn 0 --converged 0 > gpurun_out/lanes/c3_l$L.json 2> gpurun_out/lanes/c3_l$L.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/lanes/c3_l$L.json').read().strip().splitlines()[-1]); print('C3 lanes $L', round(d['value'],2), round(d['ms_per_step'],1), d['per_step']['lambda_rounds'], d['per_step']['solves_rank0'])"
done
for L in 3 4; do
  timeout -k 10 300 python3 bench.py --config C5 --no-cpu-baseline --lanes $L --steps 1 --warmup 1 --marginals 0 --search 0 --gicp 0 --live 0 --gn 0 --converged 0 > gpurun_out/lanes/c5_l$L.json 2> gpurun_out/lanes/c5_l$L.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/lanes/c5_l$L.json').read().strip().splitlines()[-1]); print('C5 lanes $L', round(d['value'],3), round(d['ms_per_step'],1), d['per_step']['lambda_rounds'], d['per_step']['solves_rank0'], d['roofline']['factorization']['frac'])"
done
