"""CPU: the PROSAC termination scan's lazy maximality updates (usac_host.hpp
ProsacTerminationCriteria, a log-free lower bound skips the candidates that cannot decide) give
the plain scan's bound and termination length on every call of random call sequences
(tests/cpp/prosac_scan_check.cpp, g++ against the host header only -- no GPU, no HIP)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_prosac_scan_lazy_equals_plain(tmp_path):
    exe = str(tmp_path / "prosac_scan_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", os.path.join(ROOT, "ransac_amd", "csrc"),
                    os.path.join(ROOT, "tests", "cpp", "prosac_scan_check.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe, "400"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr
