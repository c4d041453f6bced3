#!/bin/bash
# Round 6: the diagonal tile's factor + inverse in 8-column steps (ubench A/B,
# correctness at live sizes 64 / 37 / 8 / 1), then the new multi-rank / C5 tests.
O=gpurun_out
TAG=${TAG:-r06b}
timeout -k 10 60 ./graphslam_amd/build/ubench_factor64 > $O/${TAG}_ubench_factor64.txt 2>&1
rc=$?; cat $O/${TAG}_ubench_factor64.txt; echo "ubench rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/gpu_r06a.sh
