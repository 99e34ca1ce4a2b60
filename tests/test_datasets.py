"""Input formats and dataset front-end -- CPU checks.

Pins: every reader parses numbers as istream >> float (strtof); reading the reference's own
data files reproduces the committed golden fixtures bit for bit (those fixtures were made from
the same files by tests/golden/make_golden.py) -- skipped where /root/reference is absent; the
writers round-trip; invert3x3 == the oracle's cv::Mat::inv restatement."""
import ctypes
import os

import numpy as np
import pytest

from ransac_amd import datasets as D

REF = "/root/reference"
has_ref = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "dataset")), reason="no reference checkout")


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.int32)


def test_strtof_is_single_rounding():
    # 1.00000011920928955078125 + a hair: double rounding (via float64) and strtof differ
    s = "1.000000059604644775390625000000001"
    assert D.strtof(s) == np.nextafter(np.float32(1), np.float32(2))


def test_reader_formats_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    pts = rng.uniform(-1000, 1000, (37, 4)).astype(np.float32)
    inl = np.array([1, 5, 7, 30], np.int32)
    # LoadPointsFromFile format (SavePointsToFile writes 6 digits: compare against that rounding)
    p = tmp_path / "a_pts.txt"
    with open(p, "w") as f:
        f.write("%d\n" % len(pts))
        for r in pts:
            f.write(" ".join("%.9g" % v for v in r) + " \n")
    assert (_bits(D.load_points_from_file(p)) == _bits(pts)).all()
    D.save_points_to_file(pts, tmp_path / "b.txt", inliers=inl)
    back = D.load_points_from_file(tmp_path / "b.txt")
    assert back.shape == (4, 4) and np.allclose(back, pts[inl], rtol=1e-5)
    # x1 y1 z1 x2 y2 z2 isinlier rows
    q = tmp_path / "h_pts.txt"
    with open(q, "w") as f:
        for i, r in enumerate(pts):
            f.write("%.9g %.9g 1 %.9g %.9g 1 %d\n" % (r[0], r[1], r[2], r[3], 1 if i in inl else 0))
    p1, p2 = D.read_points(q)
    assert (_bits(np.hstack([p1, p2])) == _bits(pts)).all()
    assert D.get_inliers(q).tolist() == inl.tolist()
    # N x 6
    r6 = tmp_path / "k_vpts_pts.txt"
    with open(r6, "w") as f:
        for r in pts:
            f.write("%.9g %.9g 1 %.9g %.9g 1\n" % tuple(r))
    assert (_bits(D.get_points_nby6(r6)) == _bits(pts)).all()
    # 3x3 / 3x4 / inliers / EVD csv
    m = rng.normal(size=(3, 4)).astype(np.float32)
    (tmp_path / "m.txt").write_text("\n".join(" ".join("%.9g" % v for v in row[:3]) for row in m))
    assert (_bits(D.get_matrix3x3(tmp_path / "m.txt")) == _bits(m[:, :3])).all()
    (tmp_path / "P.txt").write_text("\n".join(" ".join("%.9g" % v for v in row) for row in m))
    assert (_bits(D.read_projection_matrix(tmp_path / "P.txt")) == _bits(m)).all()
    (tmp_path / "inl.txt").write_text("%d\n%s\n" % (len(inl), " ".join(map(str, inl))))
    assert D.read_inliers(tmp_path / "inl.txt").tolist() == inl.tolist()
    with open(tmp_path / "e.png_m.txt", "w") as f:
        f.write("x1,y1,x2,y2,FGINN_ratio,SNN_ratio,detector,descriptor,is_correct \n")
        for i, r in enumerate(pts):
            f.write("%.9g,%.9g,%.9g,%.9g,0.5,0.5,HessianAffine,RootSIFT,%d\n" % (*r, 1 if i in inl else 0))
    ep, ei = D.read_evd_points_inliers(tmp_path / "e.png_m.txt")
    assert (_bits(ep) == _bits(pts)).all() and ei.tolist() == inl.tolist()


def test_invert3x3_matches_oracle(oracle):
    rng = np.random.default_rng(3)
    L = oracle.lib()
    f32p = ctypes.POINTER(ctypes.c_float)
    for _ in range(200):
        m = rng.normal(size=9).astype(np.float32)
        out = np.zeros(9, np.float32)
        L.orc_inv3x3(m.ctypes.data_as(f32p), out.ctypes.data_as(f32p))
        assert (_bits(D.invert3x3(m)).reshape(-1) == _bits(out)).all()
    assert (D.invert3x3(np.zeros(9, np.float32)) == 0).all()


def test_dataset_lists():
    assert len(D.Dataset.getDataset(D.DATASET.Homogr_SIFT)) == 12
    assert len(D.Dataset.getDataset(D.DATASET.Kusvod2)) == 16
    assert len(D.Dataset.getDataset(D.DATASET.Syntectic)) == 8
    assert len(D.Dataset.getDataset(D.DATASET.EVD)) == 15


@has_ref
def test_reference_files_reproduce_fixtures(homography_scenes, kusvod2_scenes, line2d_scenes):
    for scene, (pts, model, _) in homography_scenes.items():
        got = D.load_points_from_file(os.path.join(REF, "dataset/homography/sift_update", scene + "_pts.txt"))
        assert (_bits(got) == _bits(pts)).all(), scene
        gm = D.get_matrix3x3(os.path.join(REF, "dataset/homography", scene + "_model.txt"))
        assert (_bits(gm).reshape(-1) == _bits(model).reshape(-1)).all(), scene
    for scene, (pts, model) in list(kusvod2_scenes.items())[:4]:
        got = D.load_points_from_file(os.path.join(REF, "dataset/Lebeda/kusvod2/sift_update", scene + "_pts.txt"))
        assert (_bits(got) == _bits(pts)).all(), scene
    for name, (pts, model, _) in line2d_scenes.items():
        got, gm, _ = D.read_line2d(os.path.join(REF, "dataset/line2d", name + ".txt"))
        assert (_bits(got) == _bits(pts)).all() and (_bits(gm) == _bits(model).reshape(-1)[:3]).all()
