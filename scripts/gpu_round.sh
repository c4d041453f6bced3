#!/bin/bash
# Full round check on the GPU box: parity tests (all), smoke, default bench, profiles.
set -o pipefail
mkdir -p gpurun_out
run() {
  local t=$1 log=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc" | tee -a gpurun_out/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
run 1200 pytest_gpu.log python -m pytest tests -m gpu -q
run 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 900 bench.log python bench.py
[ "${SKIP_PROFILE:-0}" = "1" ] || run 1500 profile.log bash scripts/gpu_profile.sh
if [ "${EXTRA:-0}" = "1" ]; then
  run 600 c5_bench.log python bench.py --config C5 --steps 1 --warmup 0 --no-cpu-baseline --marginals 0 --search 0
  # multi-GPU rehearsal on one box: 2 ranks on cuda:0 (host transport), partitioned factorisation
  run 600 part2_bench.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --multi partition --same-device --steps 2 --warmup 1 --marginals 0 --search 0
fi
echo done
