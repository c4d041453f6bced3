#!/bin/bash
# Panel chain vs plain Schur tiles A/B: hardware queues, the plain tiles' stream
# kept off some CUs (PGO_SIDE_CUMASK), the look-ahead on smaller fronts.
O=gpurun_out
timeout -k 10 900 python3 scripts/factor_breakdown.py --reps 10 --envs "hwq8:GPU_MAX_HW_QUEUES=8" \
  "cum4:PGO_SIDE_CUMASK=4" "cum4m1:PGO_SIDE_CUMASK=4,PGO_SIDE_CUMASK_MODE=1" "la512:PGO_LOOKAHEAD_M=512" \
  "cum4la:PGO_SIDE_CUMASK=4,PGO_LOOKAHEAD_M=512" "cum8la:PGO_SIDE_CUMASK=8,PGO_LOOKAHEAD_M=512" \
  "hwq8cum4la:GPU_MAX_HW_QUEUES=8,PGO_SIDE_CUMASK=4,PGO_LOOKAHEAD_M=512" "default2:PGO_DUMMY=2" > $O/r04j_ab.txt 2>&1 || { echo "ab failed"; tail -5 $O/r04j_ab.txt; exit 1; }
grep -v "^{" $O/r04j_ab.txt
