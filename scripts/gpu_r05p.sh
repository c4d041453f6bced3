#!/bin/bash
# Round 5: replay A/B of the number of hardware queues (the factor graph's
# cross-stream edges cost ~10 us of GPU idle each at 4 queues, scripts/idle_gaps.py)
O=gpurun_out
timeout -k 10 500 python3 scripts/factor_breakdown.py --config C3 --lanes 1 3 --envs "q1:GPU_MAX_HW_QUEUES=1" "q2:GPU_MAX_HW_QUEUES=2" "q3:GPU_MAX_HW_QUEUES=3" > $O/r05p_queues.txt 2>&1 || exit 1
tail -1 $O/r05p_queues.txt
echo done
