#!/bin/bash
# Round 5: Schur tile kernel with 32-column chunks (k_panel_syrk_lds32) against
# the 16-column form and the others (scripts/ubench_syrk.hip), three front sizes.
O=gpurun_out
for m in 4096 2048 1024; do
  timeout -k 10 120 ./graphslam_amd/build/ubench_syrk $m 512 > $O/r05n_syrk_$m.txt 2>&1 || { echo "ubench $m failed"; tail -3 $O/r05n_syrk_$m.txt; exit 1; }
  grep "^m " $O/r05n_syrk_$m.txt
done
echo done
