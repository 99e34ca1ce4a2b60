"""Input formats and the dataset front-end of the reference.

Readers (detector/Reader.cpp) parse numbers as ``std::istream >> float`` does -- correctly
rounded decimal-to-float (strtof), not through a double -- so the loaded points are the
reference's bit for bit:

  read_points            Reader::read_points          x1 y1 z1 x2 y2 z2 isinlier rows
  get_inliers            Reader::getInliers           the same rows -> indices with isinlier > 0
  get_matrix3x3          Reader::getMatrix3x3         3 x 3 model file
  read_projection_matrix Reader::readProjectionMatrix 3 x 4
  load_points_from_file  Reader::LoadPointsFromFile   "N" then N rows "x1 y1 x2 y2" (*_pts / *_spts)
  save_points_to_file    Reader::SavePointsToFile
  get_points_nby6        Reader::getPointsNby6        x1 y1 1 x2 y2 1 rows -> N x 4
  read_evd_points_inliers Reader::readEVDPointsInliers EVD csv (header, is_correct column)
  read_inliers           Reader::readInliers          "count" then indices

``ImageData`` mirrors dataset/GetImage.h: points, PROSAC-sorted points, GT model and the GT
inlier derivation (getGTInliers / getGTInliersSorted: Quality::getInliers of the GT model on
the device, homography also with model.inv() -- the restated cv::Mat::inv -- fundamental also
with model.t(), keeping the larger set), densitySort for the synthetic line sets (KNN
distances on the device), and the Strecha GT essential matrix from its inlier list
(EstimateModelNonMinimalSample on the device).  Images are not loaded (GUI only).
``Dataset`` holds the reference's scene lists (dataset/Dataset.cpp).
"""
import ctypes
import enum
import os

import numpy as np

_libc = ctypes.CDLL("libc.so.6")
_libc.strtof.restype = ctypes.c_float
_libc.strtof.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p)]


def strtof(tok):
    """decimal -> float, correctly rounded (what istream >> float does)."""
    return _libc.strtof(tok.encode() if isinstance(tok, str) else tok, None)


def _floats(tokens):
    return np.array([strtof(t) for t in tokens], dtype=np.float32)


def _tokens(path):
    with open(path) as f:
        return f.read().split()


class DATASET(enum.IntEnum):  # dataset/Dataset.h:12
    Homogr = 0
    Homogr_SIFT = 1
    Adelaidermf = 2
    Adelaidermf_SIFT = 3
    Kusvod2 = 4
    Kusvod2_SIFT = 5
    Syntectic = 6
    Strecha = 7
    EVD = 8


# ----------------------------------------------------------------- Reader (detector/Reader.cpp)
def read_points(path):
    """Reader::read_points (Reader.cpp:12-47): rows x1 y1 z1 x2 y2 z2 inl -> (pts1, pts2)."""
    t = _tokens(path)
    rows = len(t) // 7
    v = _floats(t[: 7 * rows]).reshape(rows, 7)
    return np.ascontiguousarray(v[:, 0:2]), np.ascontiguousarray(v[:, 3:5])


def get_inliers(path):
    """Reader::getInliers (Reader.cpp:72-118): indices of rows whose 7th value (int) is > 0."""
    t = _tokens(path)
    rows = len(t) // 7
    return np.array([p for p in range(rows) if int(t[7 * p + 6]) > 0], dtype=np.int32)


def get_matrix3x3(path):
    """Reader::getMatrix3x3 (Reader.cpp:129-145): 9 floats, row-major."""
    t = _tokens(path)
    if len(t) < 9:
        raise ValueError("Wrong direction to matrix file! (%s)" % path)
    return _floats(t[:9]).reshape(3, 3)


def read_projection_matrix(path):
    """Reader::readProjectionMatrix (Reader.cpp:263-279): 3 x 4."""
    t = _tokens(path)
    if len(t) < 12:
        raise ValueError("Wrong direction to Projection matrix file! (%s)" % path)
    return _floats(t[:12]).reshape(3, 4)


def load_points_from_file(path):
    """Reader::LoadPointsFromFile (Reader.cpp:182-213): first line N, then lines of 4 values."""
    with open(path) as f:
        lines = f.read().splitlines()
    if not lines:
        raise ValueError("empty points file %s" % path)
    n = int(lines[0].split()[0])
    out = np.zeros((n, 4), dtype=np.float32)
    r = 0
    for ln in lines[1:]:
        tok = ln.split()
        if not tok or r >= n:
            continue
        out[r, : min(4, len(tok))] = _floats(tok[:4])
        r += 1
    return out


def save_points_to_file(points, path, inliers=None):
    """Reader::SavePointsToFile (Reader.cpp:149-180): count line, then rows (all, or the inliers)."""
    pts = np.asarray(points, dtype=np.float32)
    rows = pts if inliers is None else pts[np.asarray(inliers, dtype=np.int64)]
    with open(path, "w") as f:
        f.write("%d\n" % len(rows))
        for r in rows:
            f.write("".join("%s " % _fmt(v) for v in r) + "\n")


def _fmt(v):
    """ostream << float with the default 6 significant digits."""
    return "%g" % float(v)


def get_points_nby6(path):
    """Reader::getPointsNby6 (Reader.cpp:57-66): rows x1 y1 z1 x2 y2 z2 -> N x 4 [x1 y1 x2 y2]."""
    t = _tokens(path)
    rows = len(t) // 6
    v = _floats(t[: 6 * rows]).reshape(rows, 6)
    return np.ascontiguousarray(v[:, [0, 1, 3, 4]])


def read_evd_points_inliers(path):
    """Reader::readEVDPointsInliers (Reader.cpp:215-260): csv with a header line; returns
    (points N x 4, inliers of rows whose is_correct != 0)."""
    with open(path) as f:
        lines = f.read().splitlines()
    pts, inl = [], []
    for i, ln in enumerate(x for x in lines[1:] if x.strip()):
        c = ln.split(",")
        pts.append([strtof(c[0]), strtof(c[1]), strtof(c[2]), strtof(c[3])])
        if strtof(c[8]) != 0:
            inl.append(i)
    return np.array(pts, dtype=np.float32).reshape(-1, 4), np.array(inl, dtype=np.int32)


def read_inliers(path):
    """Reader::readInliers (Reader.cpp:281-296): count, then that many indices."""
    t = _tokens(path)
    if not t:
        raise ValueError("Wrong direction to inliers file (%s)" % path)
    k = int(t[0])
    return np.array([int(x) for x in t[1: 1 + k]], dtype=np.int32)


def read_line2d(path):
    """dataset/GetImage.h:85-116 (DATASET::Syntectic): width height noise a b c N, N x (x y)."""
    t = _tokens(path)
    w, h, noise = int(t[0]), int(t[1]), int(float(t[2]))
    model = _floats(t[3:6])
    n = int(t[6])
    pts = _floats(t[7: 7 + 2 * n]).reshape(n, 2)
    return pts, model, (w, h, noise)


# ----------------------------------------------------------------- model helpers
def invert3x3(m):
    """cv::Mat::inv of a float 3 x 3 as restated for the device (usac_device.hpp:inv3x3):
    fp64 cofactors and 1/det, one cast to float; singular -> zeros."""
    a = [float(x) for x in np.asarray(m, dtype=np.float32).reshape(-1)]

    def M(r, c):
        return a[3 * r + c]

    d = (M(0, 0) * (M(1, 1) * M(2, 2) - M(1, 2) * M(2, 1)) - M(0, 1) * (M(1, 0) * M(2, 2) - M(1, 2) * M(2, 0)) +
         M(0, 2) * (M(1, 0) * M(2, 1) - M(1, 1) * M(2, 0)))
    if d == 0.0:
        return np.zeros((3, 3), dtype=np.float32)
    d = 1.0 / d
    out = [(M(1, 1) * M(2, 2) - M(1, 2) * M(2, 1)) * d, (M(0, 2) * M(2, 1) - M(0, 1) * M(2, 2)) * d,
           (M(0, 1) * M(1, 2) - M(0, 2) * M(1, 1)) * d, (M(1, 2) * M(2, 0) - M(1, 0) * M(2, 2)) * d,
           (M(0, 0) * M(2, 2) - M(0, 2) * M(2, 0)) * d, (M(0, 2) * M(1, 0) - M(0, 0) * M(1, 2)) * d,
           (M(1, 0) * M(2, 1) - M(1, 1) * M(2, 0)) * d, (M(0, 1) * M(2, 0) - M(0, 0) * M(2, 1)) * d,
           (M(0, 0) * M(1, 1) - M(0, 1) * M(1, 0)) * d]
    return np.array(out, dtype=np.float32).reshape(3, 3)


def density_sort(points, knn=13, device=0):
    """densitySort (usac/utils/utils.cpp:8-32): points ordered by the fp32 sum of their knn
    squared neighbour distances (nanoflann KNN -> usac_knn on the device), ascending.  The
    reference's std::sort leaves equal sums unordered; here they keep index order (unpinned)."""
    import ransac_amd as usac

    pts = np.ascontiguousarray(points, dtype=np.float32)
    est = usac.ESTIMATOR.Line2d if pts.shape[1] == 2 else usac.ESTIMATOR.Homography
    with usac.Context(est, pts, device=device) as ctx:
        _, d2 = ctx.knn(knn)
    s = np.zeros(len(pts), dtype=np.float32)
    for k in range(knn):  # sequential fp32 sum, column by column == per-row in order
        s = (s + d2[:, k]).astype(np.float32)
    order = np.argsort(s, kind="stable")
    return np.ascontiguousarray(pts[order]), order


# ----------------------------------------------------------------- Dataset lists
class Dataset:
    """dataset/Dataset.cpp scene lists."""

    HOMOGRAPHY = ["adam", "Brussels", "boat", "BostonLib", "city", "Boston", "Eiffel", "WhiteBoard", "BruggeSquare",
                  "ExtremeZoom", "BruggeTower", "graf"]
    HOMOGRAPHY_PROBLEM = ["LePoint1", "LePoint2", "LePoint3", "CapitalRegion"]
    KUSVOD2 = ["booksh", "box", "castle", "corr", "graff", "head", "kampa", "Kyoto", "leafs", "plant", "rotunda",
               "shout", "valbonne", "wall", "wash", "zoom"]
    ADELAIDERMF = ["bonhall", "elderhallb", "hartley", "johnsona", "johnsonb", "ladysymon", "library", "napiera",
                   "napierb", "neem", "nese", "oldclassicswing", "physics", "sene", "unihouse"]
    EVD = ["adam", "cafe", "mag", "cat", "dum", "face", "fox", "girl", "graf", "grand", "index", "pkk", "shop", "there",
           "vin"]
    LINE2D = ["w=1000_h=1000_n=3.000000_I=200_N=10200", "w=1000_h=1000_n=3.000000_I=500_N=10500",
              "w=1000_h=1200_n=3.000000_I=200_N=10200", "w=1000_h=1200_n=3.000000_I=500_N=10500",
              "w=1200_h=1000_n=3.000000_I=200_N=10200", "w=1200_h=1000_n=3.000000_I=500_N=10500",
              "w=1200_h=1200_n=3.000000_I=200_N=10200", "w=1200_h=1200_n=3.000000_I=500_N=10500"]

    @staticmethod
    def getDataset(dataset, root="."):
        d = DATASET(dataset)
        if d in (DATASET.Homogr, DATASET.Homogr_SIFT):
            return list(Dataset.HOMOGRAPHY)
        if d in (DATASET.Adelaidermf, DATASET.Adelaidermf_SIFT):
            return list(Dataset.ADELAIDERMF)
        if d in (DATASET.Kusvod2, DATASET.Kusvod2_SIFT):
            return list(Dataset.KUSVOD2)
        if d == DATASET.Syntectic:
            return list(Dataset.LINE2D)
        if d == DATASET.EVD:
            return list(Dataset.EVD)
        with open(os.path.join(root, "dataset", "MVS", "zdataset.txt")) as f:  # Strecha
            return f.read().split()


# ----------------------------------------------------------------- ImageData (GetImage.h)
class ImageData:
    """dataset/GetImage.h ImageData(dataset, img_name) with the dataset tree under `root`
    (the directory holding dataset/).  GT inlier derivation and the Strecha GT model run on
    the device."""

    def __init__(self, dataset, img_name, root=".", device=0):
        import ransac_amd as usac

        d = DATASET(dataset)
        self.dataset, self.name, self.device = d, img_name, device
        self.inliers = None
        self.sorted_inliers = None
        self.sorted_pts = None
        D = lambda *p: os.path.join(root, "dataset", *p)  # noqa: E731
        if d == DATASET.Adelaidermf:
            self.estimator = usac.ESTIMATOR.Fundamental
            p1, p2 = read_points(D("adelaidermf", img_name + "_pts.txt"))
            self.pts = np.hstack([p1, p2])
            self.inliers = get_inliers(D("adelaidermf", img_name + "_pts.txt"))
            self.model = get_matrix3x3(D("adelaidermf", img_name + "_model.txt"))
        elif d == DATASET.Adelaidermf_SIFT:
            self.estimator = usac.ESTIMATOR.Fundamental
            self.pts = load_points_from_file(D("adelaidermf", "sift_update", img_name + "_pts.txt"))
            self.sorted_pts = load_points_from_file(D("adelaidermf", "sift_update", img_name + "_spts.txt"))
            self.model = get_matrix3x3(D("adelaidermf", img_name + "_model.txt"))
        elif d == DATASET.Kusvod2:
            self.estimator = usac.ESTIMATOR.Fundamental
            self.pts = get_points_nby6(D("Lebeda", "kusvod2", img_name + "_vpts_pts.txt"))
            self.model = get_matrix3x3(D("Lebeda", "kusvod2", img_name + "_vpts_model.txt"))
        elif d == DATASET.Kusvod2_SIFT:
            self.estimator = usac.ESTIMATOR.Fundamental
            self.pts = load_points_from_file(D("Lebeda", "kusvod2", "sift_update", img_name + "_pts.txt"))
            self.sorted_pts = load_points_from_file(D("Lebeda", "kusvod2", "sift_update", img_name + "_spts.txt"))
            self.model = get_matrix3x3(D("Lebeda", "kusvod2", img_name + "_vpts_model.txt"))
        elif d == DATASET.Strecha:
            self.estimator = usac.ESTIMATOR.Essential
            self.pts = load_points_from_file(D("MVS", img_name + "_pts.txt"))
            self.sorted_pts = load_points_from_file(D("MVS", img_name + "_spts.txt"))
            self.inliers = read_inliers(D("MVS", img_name + "_inl.txt"))
            with usac.Context(self.estimator, self.pts, device=device) as ctx:
                self.model = ctx.nonminimal(self.inliers).reshape(3, 3)
            with usac.Context(self.estimator, self.sorted_pts, device=device) as ctx:
                _, _, self.sorted_inliers = ctx.get_inliers(self.model.reshape(-1), 1.0)  # threshold 1
        elif d == DATASET.Syntectic:
            self.estimator = usac.ESTIMATOR.Line2d
            self.pts, self.model, self.image_size = read_line2d(D("line2d", img_name + ".txt"))
            self.sorted_pts, _ = density_sort(self.pts, 13, device)
        elif d == DATASET.EVD:
            self.estimator = usac.ESTIMATOR.Homography
            self.pts, self.inliers = read_evd_points_inliers(D("EVD", "EVD_tentatives", img_name + ".png_m.txt"))
            self.sorted_inliers = self.inliers.copy()  # points (inliers) are already sorted
            self.sorted_pts = self.pts.copy()
            self.model = get_matrix3x3(D("EVD", "h", img_name + ".txt"))
        elif d == DATASET.Homogr_SIFT:
            self.estimator = usac.ESTIMATOR.Homography
            self.pts = load_points_from_file(D("homography", "sift_update", img_name + "_pts.txt"))
            self.sorted_pts = load_points_from_file(D("homography", "sift_update", img_name + "_spts.txt"))
            self.model = get_matrix3x3(D("homography", img_name + "_model.txt"))
        else:  # Homogr
            self.estimator = usac.ESTIMATOR.Homography
            p1, p2 = read_points(D("homography", img_name + "_pts.txt"))
            self.pts = np.hstack([p1, p2])
            self.inliers = get_inliers(D("homography", img_name + "_pts.txt"))
            self.model = get_matrix3x3(D("homography", img_name + "_model.txt"))

    # GetImage.h getters
    def getPoints(self):
        return self.pts

    def getPoints1(self):
        return np.ascontiguousarray(self.pts[:, 0:2])

    def getPoints2(self):
        return np.ascontiguousarray(self.pts[:, 2:4])

    def getSortedPoints(self):
        return self.sorted_pts

    def getModel(self):
        return self.model

    def getGTInliers(self, threshold):
        if self.inliers is None or len(self.inliers) == 0:
            self.inliers = self._gt_inliers(self.pts, threshold)
        return self.inliers

    def getGTInliersSorted(self, threshold):
        if self.sorted_inliers is None or len(self.sorted_inliers) == 0:
            self.sorted_inliers = self._gt_inliers(self.sorted_pts, threshold)
        return self.sorted_inliers

    def _gt_inliers(self, pts, thr):
        """getGTInliersFromGTModel* (GetImage.h:245-330): Quality::getInliers of the GT model;
        homography also model.inv(), fundamental also model.t(), the larger set wins (and
        replaces the model)."""
        import ransac_amd as usac

        with usac.Context(self.estimator, pts, device=self.device) as ctx:
            _, _, inl = ctx.get_inliers(self.model.reshape(-1), thr)
            alt = None
            if self.estimator == usac.ESTIMATOR.Homography:
                alt = invert3x3(self.model)
            elif self.estimator == usac.ESTIMATOR.Fundamental:
                alt = np.ascontiguousarray(self.model.T)
            if alt is not None:
                _, _, inl2 = ctx.get_inliers(alt.reshape(-1), thr)
                if len(inl2) > len(inl):
                    inl = inl2
                    self.model = alt
        return inl
