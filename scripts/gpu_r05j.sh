#!/bin/bash
# Round 5: FETCH_SIZE / WRITE_SIZE calibration for this repo's access widths
# (scripts/ubench_pmc_calib.hip), each pass a run of its own.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/calib
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1; echo "list rc=$?"
grep -oE "TCC_EA0?_(RD|WR)REQ[A-Z0-9_]*" $O/counters.txt | sort -u > $O/tcc_ea.txt || true
cat $O/tcc_ea.txt | head -40
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $c -T -f csv -d $O/$c -o calib -- ./graphslam_amd/build/ubench_pmc_calib > $O/$c.log 2>&1
  echo "pmc $c rc=$?"
done
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ TCC_EA0_RDREQ_32B -T -f csv -d $O/RDREQ -o calib -- ./graphslam_amd/build/ubench_pmc_calib > $O/RDREQ.log 2>&1
echo "pmc RDREQ rc=$?"
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_WRREQ TCC_EA0_WRREQ_64B -T -f csv -d $O/WRREQ -o calib -- ./graphslam_amd/build/ubench_pmc_calib > $O/WRREQ.log 2>&1
echo "pmc WRREQ rc=$?"
echo done
