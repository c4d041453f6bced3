#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
PGO_LIB_PATH=graphslam_amd/libpgo_kb128.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "lm_parity or c3_full or determinism" > gpurun_out/pytest_tmp.log 2>&1
rc=$?; echo "pytest kb128 rc=$rc"; tail -2 gpurun_out/pytest_tmp.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh "PGO_LIB_PATH=graphslam_amd/libpgo.so" "PGO_LIB_PATH=graphslam_amd/libpgo_kb128.so" "PGO_LIB_PATH=graphslam_amd/libpgo.so" "PGO_LIB_PATH=graphslam_amd/libpgo_kb128.so"
