#!/bin/bash
# Replay A/B of more hardware queues than HIP's default 4 (the factor graph
# runs on up to six streams), with the default twice as the noise reference.
O=gpurun_out
timeout -k 10 500 python3 scripts/factor_breakdown.py --config C3 --lanes 1 3 --envs "q6:GPU_MAX_HW_QUEUES=6" "q8:GPU_MAX_HW_QUEUES=8" "q4:GPU_MAX_HW_QUEUES=4" "q8b:GPU_MAX_HW_QUEUES=8" > $O/r05z6_queues.txt 2>&1 || exit 1
tail -1 $O/r05z6_queues.txt
