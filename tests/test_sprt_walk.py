"""The library's SPRT walk (Sprt::verify: the per-point fp64 lambda chain a word's run at a time,
plus a certificate that lets an accepted model's remaining points be counted instead of walked)
against the reference's per-point loop (Sprt::verify_plain, sprt.hpp:191-317) on random masks of
every estimator's SPRT constants: decision, count, score, pool index and history, call for call.
Host code only (g++ on tests/native/sprt_walk_check.cpp)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_sprt_walk_equals_per_point_loop(tmp_path):
    exe = str(tmp_path / "swc")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(HERE, "..", "ransac_amd", "csrc"),
                    os.path.join(HERE, "native", "sprt_walk_check.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe, "150"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("OK"), r.stdout
