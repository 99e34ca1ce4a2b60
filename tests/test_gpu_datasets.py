"""Dataset front-end on the GPU: a dataset tree written in the reference's
file formats from the committed fixtures, loaded by ImageData (dataset/GetImage.h); the GT
inlier derivation on the device reproduces the reference's published GT inlier counts
(results/homography/uniform_gc_Grid_c_sz_50.csv "GT Inl"), and densitySort equals a numpy
restatement over the oracle's KNN distances."""
import json
import os

import numpy as np
import pytest

from ransac_amd import datasets as D

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _write_pts(path, pts):
    with open(path, "w") as f:
        f.write("%d\n" % len(pts))
        for r in pts:
            f.write(" ".join("%.9g" % v for v in r) + " \n")


def test_image_data_homography_gt_inliers(tmp_path, homography_scenes):
    gt = json.load(open(os.path.join(GOLDEN, "homography_gt.json")))["gt_inliers"]
    (tmp_path / "dataset/homography/sift_update").mkdir(parents=True)
    for scene, (pts, model, _) in homography_scenes.items():
        _write_pts(tmp_path / "dataset/homography/sift_update" / (scene + "_pts.txt"), pts)
        _write_pts(tmp_path / "dataset/homography/sift_update" / (scene + "_spts.txt"), pts[::-1])
        (tmp_path / "dataset/homography" / (scene + "_model.txt")).write_text(
            "\n".join(" ".join("%.9g" % v for v in row) for row in np.asarray(model).reshape(3, 3)))
    for scene in D.Dataset.getDataset(D.DATASET.Homogr_SIFT):
        img = D.ImageData(D.DATASET.Homogr_SIFT, scene, root=str(tmp_path))
        assert (img.getPoints().view(np.int32) == homography_scenes[scene][0].view(np.int32)).all()
        inl = img.getGTInliers(2.0)
        assert len(inl) == gt[scene], scene
        assert len(img.getGTInliersSorted(2.0)) == gt[scene], scene  # same set, reversed order


def test_density_sort_line2d(tmp_path, line2d_scenes, oracle):
    name = sorted(line2d_scenes)[0]
    pts, model, _ = line2d_scenes[name]
    (tmp_path / "dataset/line2d").mkdir(parents=True)
    m = np.asarray(model).reshape(-1)
    with open(tmp_path / "dataset/line2d" / (name + ".txt"), "w") as f:
        f.write("1000 1000 3 %.9g %.9g %.9g %d\n" % (m[0], m[1], m[2], len(pts)))
        for r in pts:
            f.write("%.9g %.9g\n" % tuple(r))
    img = D.ImageData(D.DATASET.Syntectic, name, root=str(tmp_path))
    _, d2 = oracle.knn(pts, 13)
    s = np.zeros(len(pts), np.float32)
    for k in range(13):
        s = (s + d2[:, k]).astype(np.float32)
    want = pts[np.argsort(s, kind="stable")]
    assert (img.getSortedPoints().view(np.int32) == want.view(np.int32)).all()
    assert len(img.getGTInliers(10.0)) > 100
