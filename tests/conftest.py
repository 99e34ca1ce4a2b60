import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libransac_amd.so on cuda:0)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def homography_scenes():
    z = np.load(os.path.join(GOLDEN, "homography_scenes.npz"))
    gt = json.load(open(os.path.join(GOLDEN, "homography_gt.json")))
    return {s: (z[s + "_pts"], z[s + "_model"], n) for s, n in gt["gt_inliers"].items()}


@pytest.fixture(scope="session")
def line2d_scenes():
    z = np.load(os.path.join(GOLDEN, "line2d_scenes.npz"))
    st = json.load(open(os.path.join(GOLDEN, "line2d_stats.json")))
    return {k[:-4]: (z[k], z[k[:-4] + "_model"], st["stats"][k[:-4]]) for k in z.files if k.endswith("_pts")}


@pytest.fixture(scope="session")
def usac():
    import ransac_amd
    ransac_amd.lib()
    return ransac_amd


@pytest.fixture(scope="session")
def kusvod2_scenes():
    z = np.load(os.path.join(GOLDEN, "kusvod2_scenes.npz"))
    return {k[:-4]: (z[k], z[k[:-4] + "_model"]) for k in z.files if k.endswith("_pts")}
