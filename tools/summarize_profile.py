"""Summarise a profile directory (tools/profile_round.sh) into <outdir>/<tag>_summary.json.

Per kernel: the rocprofv3 --kernel-trace --stats average duration and the PMC passes' per-dispatch
averages.  Only the kernel's full-size dispatches count (round 4): the bench's
parity checks and small launches (256-sample batches, a ramp's first batches) run the same kernels
on smaller grids, which diluted the per-launch averages -- so per kernel only the dispatches with
its largest Grid_Size are averaged (trace durations too, from run_kernel_trace.csv), and the grid
size and the number of dispatches used are recorded.  HBM traffic per launch =
FETCH_SIZE*1024*2 (gfx950 reports half the bytes of wide coalesced reads: MI355X_MICROARCH.md
§HBM) + WRITE_SIZE*1024.
  python3 tools/summarize_profile.py <dir> <tag> <n_points> <batch> <outdir> [all [runs]]
(runs: the number of whole runs the profiled command made -- full-run workloads, cfg5)
"""
import collections
import csv
import json
import os
import sys


def _grid(r):
    """a dispatch's total grid size: Grid_Size (counter CSV) or X * Y * Z (kernel-trace CSV)"""
    if r.get("Grid_Size"):
        return int(r["Grid_Size"])
    g = 1
    for d in ("X", "Y", "Z"):
        g *= int(r.get("Grid_Size_" + d, 1) or 1)
    return g


ALL_GRIDS = len(sys.argv) > 6 and sys.argv[6] == "all"  # a workload of mixed batch sizes (cfg3 exact runs)


def _max_grid_rows(rows, key):
    """rows grouped by key(row); per group only the rows of the largest grid (all of them with
    the 'all' argument)."""
    g = collections.defaultdict(list)
    for r in rows:
        g[key(r)].append(r)
    out = {}
    for k, rs in g.items():
        mg = max(_grid(r) for r in rs)
        out[k] = (rs if ALL_GRIDS else [r for r in rs if _grid(r) == mg], mg, len(rs))
    return out


def main():
    src, tag = sys.argv[1], sys.argv[2]
    out = {"source": src, "kernels": {},
           "filter": "all dispatches" if ALL_GRIDS else "largest Grid_Size dispatches per kernel"}
    if len(sys.argv) > 4:  # workload shape the bench matches on (bench.py _profile_entry)
        out["workload"] = {"n_points": int(sys.argv[3]), "batch": int(sys.argv[4])}
        if len(sys.argv) > 7:
            out["workload"]["runs"] = int(sys.argv[7])
    trace = os.path.join(src, "trace", "run_kernel_trace.csv")
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    if os.path.exists(trace):
        rows = list(csv.DictReader(open(trace)))
        for k, (rs, mg, nall) in _max_grid_rows(rows, lambda r: r["Kernel_Name"]).items():
            d = [float(r["End_Timestamp"]) - float(r["Start_Timestamp"]) for r in rs]
            out["kernels"].setdefault(k, {})["trace"] = {
                "calls": len(d), "calls_all_grids": nall, "grid_size": mg, "avg_ns": sum(d) / len(d),
                "min_ns": min(d), "max_ns": max(d)}
    elif os.path.exists(stats):
        for r in csv.DictReader(open(stats)):
            out["kernels"].setdefault(r["Name"], {})["trace"] = {
                "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "min_ns": float(r["MinNs"]),
                "max_ns": float(r["MaxNs"]), "percent": float(r["Percentage"])}
    for d in sorted(os.listdir(src)):
        if not d.startswith("pmc_"):
            continue
        f = os.path.join(src, d, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        rows = list(csv.DictReader(open(f)))
        for (k, c), (rs, mg, nall) in _max_grid_rows(rows, lambda r: (r["Kernel_Name"], r["Counter_Name"])).items():
            v = [float(r["Counter_Value"]) for r in rs]
            e = out["kernels"].setdefault(k, {})
            e.setdefault("pmc", {})[c] = sum(v) / len(v)
            e.setdefault("pmc_grid", {})[c] = [mg, len(v), nall]
    for k, v in out["kernels"].items():
        p = v.get("pmc", {})
        if "FETCH_SIZE" in p or "WRITE_SIZE" in p:
            v["hbm_bytes_per_launch"] = p.get("FETCH_SIZE", 0.0) * 1024 * 2 + p.get("WRITE_SIZE", 0.0) * 1024
    outdir = sys.argv[5] if len(sys.argv) > 5 else "profiles"
    os.makedirs(outdir, exist_ok=True)
    with open(os.path.join(outdir, "%s_summary.json" % tag), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps({k[:60]: (v.get("trace", {}).get("avg_ns"), v.get("hbm_bytes_per_launch"))
                      for k, v in out["kernels"].items()}, indent=1))


if __name__ == "__main__":
    main()
