"""Host code under AddressSanitizer (CPU): tools/asan_host.sh builds
instrumented csrc/hull.cpp + csrc/kinematics.cpp and oracle/flash_oracle.c and
drives every host path the tests reach (convex hulls incl. degenerate inputs,
FK of every model, the oracle's skin / culled skin / accumulators / RBF /
raycaster) with libasan preloaded; any ASan report fails the run."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.skipif(shutil.which("gcc") is None or shutil.which("g++") is None, reason="no host compiler")
def test_host_code_under_asan():
    libasan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not os.path.isabs(libasan) or not os.path.exists(libasan):
        pytest.skip("libasan not available")
    p = subprocess.run(["bash", os.path.join(ROOT, "tools", "asan_host.sh")], capture_output=True, text=True,
                       timeout=600)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "asan host run clean" in p.stdout
