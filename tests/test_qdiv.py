"""The slab test's reciprocal division (csrc/qdiv.h) is bit-exact against IEEE a / b
inside its documented ranges (host build of the same header; runs on CPU)."""
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def test_qdiv_exact(tmp_path):
    exe = tmp_path / "qdiv_check"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-mfma", str(REPO / "tests" / "qdiv_check.c"), "-o", str(exe), "-lm"],
                   check=True)
    r = subprocess.run([str(exe), "4000000"], capture_output=True, text=True)
    print(r.stdout)
    assert r.returncode == 0, r.stdout
    assert "mismatches 0" in r.stdout
