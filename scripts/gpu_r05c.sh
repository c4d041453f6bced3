#!/bin/bash
# Round 5: C5 multi-rank cases (4-rank partition, 2 x 2 hybrid; ranks sharing
# the GPU over gloo), C5 replay time by lanes, and a hybrid bench rehearsal
# (4 ranks on one GPU, host transport).
O=gpurun_out
TAG=${TAG:-r05c}
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_multi_gpu.py -m gpu \
  -k "c5_four_ranks or (hybrid and C5)" > $O/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 scripts/factor_breakdown.py --config C5 --lanes 1 2 3 --reps 3 --envs > $O/${TAG}_lanes_C5.txt 2>&1 || { tail -5 $O/${TAG}_lanes_C5.txt; exit 1; }
tail -1 $O/${TAG}_lanes_C5.txt
timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 4 --same-device --multi hybrid --groups 2 --steps 1 --warmup 1 --no-cpu-baseline --c5 0 --live 0 \
  --gicp 0 --search 0 --marginals 0 --gn 0 --converged 0 --profile-every 0 > $O/${TAG}_hybrid_bench.json 2> $O/${TAG}_hybrid_bench.err \
  || { echo "hybrid bench failed"; tail -5 $O/${TAG}_hybrid_bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/${TAG}_hybrid_bench.json').read().strip().splitlines()[-1]); print('hybrid bench', d['value'], d['ms_per_step'], d['config']['parallelism'], d['per_step']['final_error'])"
echo done
