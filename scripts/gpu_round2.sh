#!/bin/bash
# Round part 2 on the GPU box: rocprofv3 evidence (C3 kernel trace + PMC passes),
# GICP kernel trace, C5 bench, 2-rank partitioned rehearsal on one device.
set -o pipefail
mkdir -p gpurun_out
run() {
  local t=$1 log=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc" | tee -a gpurun_out/steps2.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
run 700 profile.log bash scripts/gpu_profile.sh
run 300 gicp_round.log bash scripts/gpu_gicp.sh
run 420 c5_bench.log python -u bench.py --config C5 --steps 1 --warmup 0 --no-cpu-baseline --marginals 0 --search 0 --live 0 --gicp 0
run 400 part2_bench.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --multi partition --same-device --steps 2 --warmup 1 --marginals 0 --search 0 --live 0 --gicp 0
echo done
