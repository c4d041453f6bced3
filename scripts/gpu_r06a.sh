#!/bin/bash
# Round 6, first GPU run: the new and changed multi-rank tests (8-rank hybrids
# on the layouts --multi auto picks, the partitioned poisoned-workspace check,
# hand-off retry / transport asserts), C5 past its first linearisation, the ABI.
O=gpurun_out
TAG=${TAG:-r06a}
timeout -k 10 1100 python -u -m pytest -x -v --timeout 900 --timeout-method thread --durations=0 \
  tests/test_abi.py tests/test_gpu_parity.py::test_c5_five_linearisations_against_fixture \
  "tests/test_multi_gpu.py::test_hybrid_matches_one_rank" tests/test_multi_gpu.py::test_partitioned_poisoned_workspace_bitwise \
  -m gpu > $O/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -30 $O/${TAG}_tests.log
exit $rc
