"""C-ABI library checks that need no GPU: it loads, exports every symbol the header
declares, and its host-side logic (sampler stream, termination, record merge) matches
the oracle."""
import ctypes
import os
import re

import numpy as np
import pytest

from tests.conftest import ROOT


def _header_functions():
    txt = open(os.path.join(ROOT, "include", "usac_gpu.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(usac_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol(usac):
    L = usac.lib()
    names = _header_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert sorted(usac.ABI_SYMBOLS) == names
    hdr = open(os.path.join(ROOT, "include", "usac_gpu.h")).read()
    assert L.usac_abi_version() == int(re.search(r"#define USAC_ABI_VERSION (\d+)", hdr).group(1))


def test_create_fails_loudly_without_gpu_or_bad_args(usac):
    with pytest.raises(Exception):
        usac.Context(usac.ESTIMATOR.Fundamental, np.zeros((10, 4), np.float32))
    with pytest.raises(Exception):
        usac.Context(usac.ESTIMATOR.Homography, np.zeros((10, 2), np.float32))


def test_host_sampler_stream_matches_oracle(usac, oracle):
    for seed, n, m in [(1, 153, 4), (7, 10000, 4), (3, 5, 4), (11, 1000, 2), (2, 9, 7)]:
        a = usac.uniform_samples(seed, n, m, 300)
        b = oracle.uniform_samples(seed, n, m, 300)
        np.testing.assert_array_equal(a, b)


def test_host_termination_matches_oracle(usac, oracle):
    for n in (153, 1000, 10000, 100000):
        for m in (2, 4, 5, 7):
            for p in (0.95, 0.99):
                for inl in np.unique(np.linspace(0, n, 97).astype(int)):
                    assert usac.std_termination(int(inl), n, m, p) == oracle.std_termination(int(inl), n, m, p)


def test_merge_records_total_order(usac):
    R = usac.Record
    recs = [R(5, 10, 3.0, (ctypes.c_float * 9)(), 1), R(2, 10, 3.0, (ctypes.c_float * 9)(), 1),
            R(1, 9, 99.0, (ctypes.c_float * 9)(), 1), R(0, 0, 0.0, (ctypes.c_float * 9)(), 0)]
    best = usac.merge_records(recs)
    assert best.hyp_index == 2 and best.inliers == 10
    recs.append(R(9, 10, 3.5, (ctypes.c_float * 9)(), 1))
    assert usac.merge_records(recs).hyp_index == 9


def test_cpp_consumer_compiles_and_links(usac):
    """include/usac_gpu.hpp (the usac_gpu:: plugin layer) compiles with g++ -std=c++11 -Werror in
    a reference-style consumer that links libransac_amd.so; its ABI check needs no GPU."""
    import json
    import subprocess

    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")], check=True)
    r = subprocess.run([os.path.join(ROOT, "tests", "cpp", "build", "consumer"), "abi"], capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout)
    assert d["abi"] == d["header"] == usac.lib().usac_abi_version()


def test_random_handle_is_the_glibc_stream(usac, oracle):
    """usac_random (the reference's global random() after srandom(seed)) needs no GPU."""
    for seed in (1, 7, 123456):
        with usac.RandomGenerator(seed) as r:
            got = [r.next() for _ in range(500)]
        assert got == oracle.glibc_stream(seed, 500).tolist()
    with usac.RandomGenerator(1) as r:
        assert [r.next(), r.next()] == [1804289383, 846930886]  # glibc KAT
