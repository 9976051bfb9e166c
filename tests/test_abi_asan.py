"""The C ABI's host code (population / DenseNet planners, workspace queries,
argument checks) under AddressSanitizer, no GPU: scripts/asan_abi.sh builds
libmpo.so with host-only ASan (-Xarch_host -fsanitize=address) and runs
tests/asan/abi_driver.cpp against it.  SURVEY §5's sanitizer item; GPU ASan is
not available on this pool."""
import os
import shutil
import subprocess

import pytest

from tests.conftest import ROOT


@pytest.mark.timeout(900)
@pytest.mark.skipif(not shutil.which("/opt/rocm/bin/hipcc") and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not installed")
def test_abi_host_code_is_asan_clean():
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "asan_abi.sh")], capture_output=True, text=True,
                       timeout=850)
    out = r.stdout + r.stderr
    assert "ERROR: AddressSanitizer" not in out, out[-4000:]
    assert r.returncode == 0 and "abi_driver: ok" in out, out[-4000:]
