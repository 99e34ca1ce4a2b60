"""Regenerate the committed golden fixtures from the reference's own data files.

Run in the build container (needs /root/reference, read-only):  python tests/golden/make_golden.py

Fixtures are DATA only -- inputs and expected outputs the reference already holds:
  * homography_scenes.npz : the 12 SIFT correspondence sets the reference's homography
    experiments use (dataset/homography/sift_update/<scene>_pts.txt, loaded as
    Reader::LoadPointsFromFile does -- detector/Reader.cpp:182-213, istream >> float,
    i.e. strtof) and their GT models (dataset/homography/<scene>_model.txt,
    Reader::getMatrix3x3, detector/Reader.cpp:129-145);
  * homography_gt.json    : the reference's published GT inlier counts for those scenes
    at threshold 2 ("GT Inl" column of results/homography/uniform_gc_Grid_c_sz_50.csv),
    derived by dataset/GetImage.h:209-231 from the GT model;
  * line2d_scenes.npz     : the synthetic line sets dataset/line2d/<name>.txt
    (format dataset/GetImage.h:85-116) and GT lines;
  * line2d_stats.json     : the published 50-run statistics of Uniform sampling on them
    (results/line2d/uniform_000.csv, thr 10, p 0.99, no LO/SPRT);
  * kusvod2_scenes.npz    : the 16 kusvod2 SIFT correspondence sets of the reference's
    fundamental experiments (dataset/Lebeda/kusvod2/sift_update/<scene>_pts.txt, the
    DATASET::Kusvod2_SIFT branch of dataset/GetImage.h:56-66) and their GT F
    (<scene>_vpts_model.txt).  The "GT Inl" column of results/kusvod2/*.csv is NOT
    reproducible from these files with the Sampson error at thr 2 (e.g. booksh: published
    149, F/F^T give 61/4), so it is not a fixture; the scenes serve as real-data inputs;
  * evd_scenes.npz        : the 15 EVD tentative correspondence sets (homography; the
    reference's EVD statistics are graph-cut runs with KNN or grid neighbours);
  * reference_stats.json  : every per-scene row (averages, standard deviations, medians) and
    the run settings of the reference's published statistical CSVs the pin tests use
    (results/line2d/{uniform,napsac,prosac}_*.csv, results/homography/uniform_gc*_Grid_c_sz_50.csv,
    results/kusvod2/uniform_gc*_Grid_c_sz_50.csv, results/EVD/*_gc*_c_sz_50.csv) -- numbers copied
    from the CSVs, nothing else.
"""
import csv
import ctypes
import json
import os

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
_libc = ctypes.CDLL("libc.so.6")
_libc.strtof.restype = ctypes.c_float
_libc.strtof.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_char_p)]


def strtof(tok):
    return _libc.strtof(tok.encode(), None)


def load_pts(path):
    with open(path) as f:
        lines = f.read().splitlines()
    n = int(lines[0])
    rows = []
    for ln in lines[1:]:
        toks = ln.split()
        if len(toks) < 4:
            continue
        rows.append([strtof(t) for t in toks[:4]])
    arr = np.array(rows, dtype=np.float32)
    assert arr.shape[0] == n, (path, arr.shape, n)
    return arr


def load_model(path):
    with open(path) as f:
        toks = f.read().split()
    return np.array([strtof(t) for t in toks[:9]], dtype=np.float32)


def homography():
    csv_path = os.path.join(REF, "results/homography/uniform_gc_Grid_c_sz_50.csv")
    gt = {}
    with open(csv_path) as f:
        for row in csv.reader(f):
            if len(row) > 2 and row[0] and row[0] != "Filename" and row[1].strip().isdigit():
                gt[row[0]] = int(row[1])
    arrays = {}
    for scene in sorted(gt):
        arrays[scene + "_pts"] = load_pts(os.path.join(REF, "dataset/homography/sift_update", scene + "_pts.txt"))
        arrays[scene + "_model"] = load_model(os.path.join(REF, "dataset/homography", scene + "_model.txt"))
    np.savez_compressed(os.path.join(OUT, "homography_scenes.npz"), **arrays)
    with open(os.path.join(OUT, "homography_gt.json"), "w") as f:
        json.dump({"source": "results/homography/uniform_gc_Grid_c_sz_50.csv (GT Inl)", "threshold": 2.0,
                   "gt_inliers": gt}, f, indent=1, sort_keys=True)


def line2d():
    arrays = {}
    names = []
    d = os.path.join(REF, "dataset/line2d")
    for fn in sorted(os.listdir(d)):
        if not fn.endswith(".txt") or fn == "dataset.txt":
            continue
        name = fn[:-4]
        with open(os.path.join(d, fn)) as f:
            toks = f.read().split()
        w, h, noise = int(toks[0]), int(toks[1]), int(toks[2])
        a, b, c = (strtof(t) for t in toks[3:6])
        n = int(toks[6])
        vals = np.array([strtof(t) for t in toks[7:7 + 2 * n]], dtype=np.float32).reshape(n, 2)
        arrays[name + "_pts"] = vals
        arrays[name + "_model"] = np.array([a, b, c], dtype=np.float32)
        names.append(name)
    np.savez_compressed(os.path.join(OUT, "line2d_scenes.npz"), **arrays)
    stats = {}
    with open(os.path.join(REF, "results/line2d/uniform_000.csv")) as f:
        rows = list(csv.reader(f))
    header = None
    for row in rows:
        if row and row[0] == "Filename":
            header = row
            continue
        if header and row and row[0] in names:
            rec = dict(zip(header, row))
            stats[row[0]] = {
                "avg_inliers": float(rec["Avg num inl/gt"].split("/")[0]),
                "std_inliers": float(rec["Std dev num inl"]),
                "avg_iters": float(rec["Avg num iters"]),
                "std_iters": float(rec["Std dev num iters"]),
                "med_iters": float(rec["Med num iters"]),
            }
    with open(os.path.join(OUT, "line2d_stats.json"), "w") as f:
        json.dump({"source": "results/line2d/uniform_000.csv", "runs": 50, "threshold": 10.0,
                   "desired_prob": 0.99, "stats": stats}, f, indent=1, sort_keys=True)


def kusvod2():
    d = os.path.join(REF, "dataset/Lebeda/kusvod2")
    scenes = sorted(fn[:-len("_pts.txt")] for fn in os.listdir(os.path.join(d, "sift_update"))
                    if fn.endswith("_pts.txt") and not fn.endswith("_spts.txt"))
    arrays = {}
    for scene in scenes:
        arrays[scene + "_pts"] = load_pts(os.path.join(d, "sift_update", scene + "_pts.txt"))
        arrays[scene + "_model"] = load_model(os.path.join(d, scene + "_vpts_model.txt"))
    np.savez_compressed(os.path.join(OUT, "kusvod2_scenes.npz"), **arrays)


def evd():
    """evd_scenes.npz: the EVD tentative correspondences (dataset/EVD/EVD_tentatives/<scene>.png_m.txt,
    Reader::readEVDPointsInliers, detector/Reader.cpp:215-260: csv after a header line, strtof)
    of the 15 scenes of results/EVD/*.csv, in file order (the reference's sorted_points for
    PROSAC are the same points: dataset/GetImage.h:122-136)."""
    d = os.path.join(REF, "dataset/EVD/EVD_tentatives")
    scenes = sorted(fn[:-len(".png_m.txt")] for fn in os.listdir(d) if fn.endswith(".png_m.txt"))
    arrays = {}
    for scene in scenes:
        with open(os.path.join(d, scene + ".png_m.txt")) as f:
            lines = [ln for ln in f.read().splitlines()[1:] if ln.strip()]
        arrays[scene + "_pts"] = np.array([[strtof(t) for t in ln.split(",")[:4]] for ln in lines], dtype=np.float32)
    np.savez_compressed(os.path.join(OUT, "evd_scenes.npz"), **arrays)


STAT_FILES = [
    "line2d/uniform_000.csv", "line2d/uniform_001.csv", "line2d/uniform_010.csv", "line2d/uniform_100.csv",
    "line2d/napsac_000.csv", "line2d/prosac_000.csv",
    "homography/uniform_gc_Grid_c_sz_50.csv", "homography/uniform_gc_sprt_Grid_c_sz_50.csv",
    "kusvod2/uniform_gc_Grid_c_sz_50.csv", "kusvod2/uniform_gc_sprt_Grid_c_sz_50.csv",
    # EVD: only the graph-cut runs hold rows (uniform_lo / uniform_sprt / prosac_lo ... are headers only)
    "EVD/uniform_gc_Nanoflann_c_sz_50.csv", "EVD/uniform_gc_sprt_Nanoflann_c_sz_50.csv",
    "EVD/prosac_gc_Nanoflann_c_sz_50.csv", "EVD/prosac_gc_sprt_Nanoflann_c_sz_50.csv",
    "EVD/prosac_gc_sprt_Grid_c_sz_50.csv",
]


def _num(v):
    v = v.strip()
    try:
        return float(v.split("/")[0]) if "/" in v else float(v)
    except ValueError:
        return v


def reference_stats():
    """tests/golden/reference_stats.json: the rows of the reference's statistical CSVs
    (written by test/tests.h getStatisticalResults + store_results_*)."""
    out = {}
    for rel in STAT_FILES:
        with open(os.path.join(REF, "results", rel)) as f:
            rows = list(csv.reader(f))
        settings, header, scenes = {}, None, {}
        for row in rows:
            if not row or not row[0].strip():
                continue
            if row[0] == "Filename":
                header = row
                continue
            if header is None:
                if " = " in row[0]:
                    k, v = row[0].split(" = ", 1)
                    settings[k.strip()] = _num(v)
                continue
            scenes[row[0]] = {h: _num(v) for h, v in zip(header[1:], row[1:])}
        out[rel] = {"settings": settings, "scenes": scenes}
    with open(os.path.join(OUT, "reference_stats.json"), "w") as f:
        json.dump({"source": "/root/reference/results (reference's published statistics)", "files": out}, f,
                  indent=1, sort_keys=True)


if __name__ == "__main__":
    reference_stats()
    homography()
    line2d()
    kusvod2()
    evd()
    print("golden fixtures written to", OUT)
