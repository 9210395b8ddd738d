"""zasr.dropin.install against the reference's real `core` modules (build container only:
the reference tree is absent on the GPU box, where this test skips).  The check itself is
tests/golden/check_dropin_install.py, run in fresh interpreters with both sys.path orders."""
import os
import subprocess
import sys

import pytest

REF = "/root/reference"
SCRIPT = os.path.join(os.path.dirname(__file__), "golden", "check_dropin_install.py")


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "core")), reason="reference tree absent")
def test_install_rebinds_reference_modules():
    r = subprocess.run([sys.executable, SCRIPT, REF], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("dropin install ok") == 2, r.stdout
    # the reference's unchanged TranscriberPipeline reaches ONE batched decode of its plan
    assert "pipeline dispatch ok" in r.stdout, r.stdout
