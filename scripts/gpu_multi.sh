#!/bin/bash
# GPU check of the multi-rank path on a one-GPU box: multi-rank parity tests
# (ranks share cuda:0 over the host transport), the whole GPU suite, and a
# 2-rank bench rehearsal (--same-device).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 ${T_TEST:-600} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_multi.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_multi.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 2 --warmup 1 --same-device --no-cpu-baseline --marginals 0 > gpurun_out/bench_spec2.log 2>&1
rc=$?; echo "bench spec2 rc=$rc"; grep '^{' gpurun_out/bench_spec2.log | cut -c1-400
exit $rc
