#!/bin/bash
# Small fronts: the trailing update one column block ahead for m > 64
# (k_front_wave, two rows per lane) and the two-wave kernel's inverse on its
# last wave ahead of its trailing share -- old / new ubench (no phase stamps;
# fingerprints must match), replay times, then the GPU test suite.
set -o pipefail
O=gpurun_out/r05u_wave.txt
: > $O
CFGS=("1 64 8" "12288 64 8" "1 100 8" "256 100 8" "2400 100 8" "1 100 16" "256 100 16" "4096 100 16" "1 64 32")
W2=("1 100 16" "256 100 16" "1 128 32" "256 128 32" "1800 128 32" "5400 128 32")
for v in oldnc nc; do
  echo "== $v" >> $O
  for cfg in "${CFGS[@]}"; do timeout -k 5 60 ./graphslam_amd/build/ubench_wave_$v $cfg >> $O || exit 1; done
  echo "== $v two waves" >> $O
  for cfg in "${W2[@]}"; do UB_WAVE2=1 timeout -k 5 60 ./graphslam_amd/build/ubench_wave_$v $cfg >> $O || exit 1; done
done
grep -E "^==|^fronts|fingerprint" $O | paste - - | head -80
timeout -k 10 300 python3 scripts/factor_breakdown.py --config C3 --lanes 1 3 --envs "small:PGO_ABLATE=small" > gpurun_out/r05u_replay.txt 2>&1 || exit 1
tail -1 gpurun_out/r05u_replay.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05u_tests.log 2>&1 || { tail -30 gpurun_out/r05u_tests.log; exit 1; }
tail -3 gpurun_out/r05u_tests.log
grep -E "C3 vs numpy|C3 solver" gpurun_out/r05u_tests.log || true
