#!/bin/bash
# Round 6: the observed differences the parity tests print (-s), to size their tolerances.
O=gpurun_out
TAG=${TAG:-r06t}
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py::test_c3_gauss_newton_against_golden tests/test_gpu_parity.py::test_c3_full_size_against_golden \
  tests/test_gpu_parity.py::test_c3_whole_trajectory_vs_numpy_twin tests/test_gpu_parity.py::test_c3_first_two_linearisations_vs_numpy_twin \
  tests/test_gpu_parity.py::test_c5_five_linearisations_against_fixture > $O/${TAG}_diffs.log 2>&1
rc=$?; grep -E "rel diff|PASSED|FAILED|passed|failed" $O/${TAG}_diffs.log; exit $rc
