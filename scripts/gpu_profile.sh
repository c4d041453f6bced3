#!/bin/bash
# rocprofv3 evidence for the bench's dominant kernels (run on the GPU box).
#   1. kernel trace + stats of the default C3 bench step (timing pass; eager
#      launches, one lambda lane: every Schur-update launch has the shape of
#      the bench's profiled factorisations, so the averages compare)
#   2. PMC passes (FETCH_SIZE, WRITE_SIZE separately) on the first linearisation
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/trace -o c3 -- \
  python3 bench.py --config C3 --steps 1 --warmup 1 --no-cpu-baseline --no-graphs --lanes 1 --live 0 --gicp 0 --search 0 --marginals 0 --c5 0 > $OUT/trace_bench.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
find $OUT/trace -name "*kernel_trace.csv" -exec gzip -f {} \;
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c -T -f csv -d $OUT/pmc_$c -o c3 \
    --kernel-include-regex "k_step|k_panel_first|k_panel_syrk|k_assemble_tile|k_front_wave|k_bwd_part|k_linearize|k_pcg_spmv" -- \
    python3 bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-graphs --lanes 1 --max-outer 1 --live 0 --gicp 0 --search 0 --marginals 0 --c5 0 > $OUT/pmc_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  find $OUT/pmc_$c -name "*counter_collection.csv" -exec gzip -f {} \;
done
echo done
