"""Host AddressSanitizer + UBSan run of the C-ABI ("-fsanitize=
address,undefined build of the C-ABI layer run against the CPU path").

`make -C slam-robot_simu_amd asan` builds libslam_hip_asan.so with every TU's
host side instrumented (device code unchanged) and tests/asan/capi_asan_driver
.cpp against it, then runs the driver: every entry point's argument checks and
error returns (NULL handles and arguments, bad sizes, creates with no device)
and the host-only paths (MT19937 jump-ahead against the recurrence, the glibc
log restatement against this process's log(), the shard split).  A sanitizer
report aborts the driver, failing the test.  No GPU needed."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "slam-robot_simu_amd")


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="no hipcc")
def test_capi_under_asan_ubsan():
    r = subprocess.run(["make", "-C", PKG, "-j", str(min(8, os.cpu_count() or 4)), "asan"],
                       capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "0 failed" in out, out[-2000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
