#!/bin/bash
O=gpurun_out
timeout -k 10 60 ./graphslam_amd/build/ubench_factor64 > $O/${TAG}_ubench_factor64.txt 2>&1
rc=$?; cat $O/${TAG}_ubench_factor64.txt; echo "ubench rc=$rc"
if [ -x ./graphslam_amd/build/ubench_d8parts ]; then
  timeout -k 10 60 ./graphslam_amd/build/ubench_d8parts > $O/${TAG}_ubench_d8parts.txt 2>&1
  echo "parts rc=$?"; cat $O/${TAG}_ubench_d8parts.txt
fi
