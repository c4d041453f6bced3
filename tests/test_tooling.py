"""SURVEY.md §5 tooling: host sanitizer builds and roctx ranges.

* The C restatement (oracle/) built with AddressSanitizer + UndefinedBehavior-
  Sanitizer and driven through every entry point by oracle/selftest.c.
* libpgo's host planning code (symbolic analysis, orderings, partition,
  incremental paths) built the same way (hipcc -Xarch_host) and driven by
  graphslam_amd/csrc/host_selftest.cpp -- host code only, no GPU.
* libpgo.so carries roctx ranges (pgo_optimize > plan / linearisation >
  lambda_round) for rocprofv3 --marker-trace.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(cmd, timeout=300, env=None):
    return subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=env)


def test_oracle_under_asan_ubsan():
    b = _run(["make", "-s", "-C", "oracle", "sanitize"])
    assert b.returncode == 0, b.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="halt_on_error=1")
    r = _run([os.path.join(ROOT, "oracle", "build", "selftest_asan")], env=env)
    assert r.returncode == 0 and "selftest ok" in r.stdout, (r.stdout + r.stderr)[-3000:]


@pytest.mark.parametrize("xcd_order", ["1", "2"])
def test_planner_under_asan_ubsan(xcd_order):
    """xcd_order 2: the tile-assembly tasks of every level dealt to the XCDs
    (the default does it only on levels of >= 2048 tiles, none in the self-test's
    graphs) -- the assembly checks then see the reordered lists."""
    b = _run(["make", "-s", "-C", "graphslam_amd/csrc", "asan-host"], timeout=600)
    assert b.returncode == 0, b.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="halt_on_error=1", PGO_ASM_XCD=xcd_order,
               PGO_SELFTEST_QUICK="1" if xcd_order == "2" else "0")
    r = _run([os.path.join(ROOT, "graphslam_amd", "csrc", "build", "host_selftest_asan")], env=env)
    assert r.returncode == 0 and "host selftest ok" in r.stdout, (r.stdout + r.stderr)[-3000:]


def test_libpgo_has_roctx_ranges(pgo_lib):
    from graphslam_amd import _lib
    r = _run(["nm", "-D", _lib.LIB_PATH])
    if r.returncode != 0:
        pytest.skip("nm unavailable")
    assert "roctxRangePushA" in r.stdout and "roctxRangePop" in r.stdout
