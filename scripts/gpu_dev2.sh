#!/bin/bash
# Development check on the GPU box: all parity tests, smoke, a quick C3 bench,
# the backward-solve timeline of one profiled factorisation, and a kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {
  local t=$1 log=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "[$log] rc=$rc" | tee -a gpurun_out/steps_dev.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
run 600 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()"
run 300 qb.log python3 bench.py --no-cpu-baseline --live 0 --gicp 0 --search 0 --marginals 0
[ -f graphslam_amd/libpgo_b.so ] && run 700 ab_run.log bash scripts/gpu_ab_lib.sh
rm -f gpurun_out/dump.txt
PGO_PROFILE_DUMP=gpurun_out/dump.txt run 300 dump_bench.log python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --live 0 --gicp 0 --search 0 --marginals 0
python3 scripts/bwd_timeline.py gpurun_out/dump.txt 1 > gpurun_out/bwd_timeline.txt 2>&1
[ "${TRACE:-1}" = "1" ] && TAG=dev bash scripts/gpu_trace.sh
echo done
