"""The step kernel's Box-Muller angle (qcart_kernels.hpp sincospi_unit: sin/cos(pi t) by exact reduction to
|r| <= 1/4 and Taylor kernels) restated operation for operation in C (tools/sincospi_check.c, fma/rint as on the
device) and checked against long double on the host: within 3e-16 of the exact sin/cos(2 pi u2), i.e. at least
as close as the oracle's libm on the rounded 2 pi u2."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_box_muller_angle_within_3e16_of_exact(tmp_path):
    exe = tmp_path / "sincospi_check"
    subprocess.check_call(["gcc", "-O2", "-o", str(exe), os.path.join(ROOT, "tools", "sincospi_check.c"), "-lm"])
    out = subprocess.check_output([str(exe), "2000000"], text=True)
    m = re.search(r"mine vs exact: sin (\S+) cos (\S+); libm\(2pi u2 rounded\) vs exact (\S+)", out)
    assert m, out
    es, ec, el = (float(x) for x in m.groups())
    assert es < 3e-16 and ec < 3e-16, out
    assert max(es, ec) <= el, out              # no worse than the oracle's own libm path
    assert "t=.5: 1 -0" in out                 # exact quadrant point: sin(pi/2) = 1, cos = -0
