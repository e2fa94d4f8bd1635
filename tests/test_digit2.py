"""The short two-level digit form (Digit2, csrc/pbs_common.h) and the one-level DigitL1 against
decomp_digit32: 2^24 hi words per base log (1..15 / 1..30) (the full 2^32 sweep: scripts/check_digit2.cpp without an argument)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_digit2_matches_decomp_digit32(tmp_path):
    exe = str(tmp_path / "check_digit2")
    subprocess.run(["g++", "-O2", "-fopenmp", os.path.join(ROOT, "scripts", "check_digit2.cpp"), "-o", exe], check=True)
    out = subprocess.run([exe, "24"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.count("mismatches 0") == 15 + 30
