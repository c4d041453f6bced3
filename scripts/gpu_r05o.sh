#!/bin/bash
# Round 5: kernel trace of the default C3 optimize (graph replays, 3 lambda lanes,
# no per-launch profiling step) to measure the GPU's idle time between and inside
# the lambda rounds (scripts/idle_gaps.py).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05o
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace -T -f csv -d $O/trace -o c3 -- \
  python3 bench.py --config C3 --steps 1 --warmup 1 --profile-every 0 --no-cpu-baseline --live 0 --gicp 0 --search 0 --marginals 0 --c5 0 --gn 0 --converged 0 > $O/bench.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/bench.log; exit $rc; }
find $O/trace -name "*kernel_trace.csv" -exec gzip -f {} \;
echo done
