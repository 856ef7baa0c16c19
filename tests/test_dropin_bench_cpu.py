"""tools/bench_dropin.py's process model on the CPU kind (the oracle processes, no GPU): every family at its driver
defaults, with the driver's per-interval call, counts calls inside the common window."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("family,extra", [("inverted_quartic", ["--driver-loop"]), ("quartic", ["--driver-loop"]),
                                          ("harmonic", ["--n-max", "70"]), ("inverted_harmonic", ["--driver-loop"])])
def test_bench_dropin_cpu_kind(tmp_path, family, extra):
    out = tmp_path / "r.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "bench_dropin.py"), "--procs", "2", "--kinds", "cpu",
                    "--seconds", "0.6", "--family", family, "--out", str(out)] + extra,
                   cwd=ROOT, check=True, timeout=300, capture_output=True)
    r = json.load(open(out))
    assert r["family"] == family and len(r["rows"]) == 1
    row = r["rows"][0]
    assert row["kind"] == "cpu" and row["procs"] == 2 and row["step_calls_per_s"] > 0
    assert row["driver_loop"] == ("--driver-loop" in extra)
