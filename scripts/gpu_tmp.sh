timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_graph.log 2>&1; echo "bench rc=$?"; TAG=chol3 bash scripts/gpu_trace.sh
