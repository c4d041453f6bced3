#!/bin/bash
# GPU-box run: parity tests, smoke, short benches.  Stops at the first GPU step
# that times out / aborts / segfaults (rc not in {0,1}).
set -o pipefail
mkdir -p gpurun_out
(lscpu | head -20; nproc; rocminfo | grep -m3 gfx) > gpurun_out/box.txt 2>&1
run() {  # run <timeout> <log> <cmd...>
  local t=$1 log=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc" | tee -a gpurun_out/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
run 900 pytest_gpu.log python -m pytest tests -m gpu -q -k "${PYTEST_K:-not c3}"
run 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 300 bench_c2.log python bench.py --config C2 --steps 2 --warmup 1 --no-cpu-baseline
run 600 bench_c3.log python bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline
echo done
