#!/bin/bash
# Round 5: read-request sizes behind FETCH_SIZE (64-B vs 128-B requests) for the
# calibration kernels, then the same counters on the C3 bench's first
# linearisation (exact read bytes = 64 RDREQ_64B + 128 RDREQ_128B + 32 RDREQ_32B).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/calib2
mkdir -p $O
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B -T -f csv -d $O/REQSZ -o calib -- ./graphslam_amd/build/ubench_pmc_calib > $O/REQSZ.log 2>&1
echo "pmc REQSZ rc=$?"
for c in "TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B" "TCC_EA0_RDREQ_32B TCC_EA0_RDREQ" WRITE_SIZE; do
  tag=$(echo $c | tr ' ' '_')
  timeout -k 10 600 rocprofv3 --pmc $c -T -f csv -d $O/c3_$tag -o c3 \
    --kernel-include-regex "k_step|k_panel_first|k_panel_syrk|k_assemble_tile|k_vec_assemble|k_front_wave|k_bwd_part|k_linearize" -- \
    python3 bench.py --config C3 --steps 1 --warmup 0 --no-cpu-baseline --no-graphs --lanes 1 --max-outer 1 --live 0 --gicp 0 --search 0 --marginals 0 --c5 0 > $O/c3_$tag.log 2>&1
  rc=$?; echo "pmc c3 $tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
echo done
