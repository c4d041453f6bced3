#!/bin/bash
# Round 6: the whole GPU suite and smoke on the default build (forward-
# substitution diagonal tiles), then a 4-rank bench rehearsal on the shared
# device (host transport; --multi auto: the model's choice, the agreement-point
# setup path) -- its time means nothing, its final error must be one GPU's.
O=gpurun_out
TAG=${TAG:-r06d}
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread --durations=15 tests -m gpu > $O/${TAG}_pytest_gpu.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -22 $O/${TAG}_pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; cat $O/${TAG}_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 4 --same-device --config C2 --steps 1 --warmup 1 --c5 0 --live 0 --gicp 0 --marginals 0 --search 0 > $O/${TAG}_rehearsal4.json 2> $O/${TAG}_rehearsal4.err
rc=$?; echo "rehearsal rc=$rc"; tail -3 $O/${TAG}_rehearsal4.err
python3 -c "import json; d=json.loads(open('$O/${TAG}_rehearsal4.json').read().strip().splitlines()[-1]); print(d['config']['parallelism'], d['config']['multi_mode'][:120], d['per_step']['final_error'], d['per_step']['transport'], d['per_step']['handoff_retries'])"
echo done
