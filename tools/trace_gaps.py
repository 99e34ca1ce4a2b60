"""Inter-kernel gaps of a rocprofv3 kernel trace (run_kernel_trace.csv): per stream, consecutive
dispatches sorted by start; gap = start - previous end (the dependent-launch latency the device
adds between kernels of one stream).  Prints the kernel / gap totals and the median gap, overall
and for the kernels named by a filter (default: the LO / polish stage kernels of cfg5).
  python3 tools/trace_gaps.py <run_kernel_trace.csv> [substring ...]
"""
import collections
import csv
import json
import statistics
import sys

LO = ("k_gather_psum4", "k_seq_seg", "k_seq_link", "k_seq_psum", "k_norm_dist", "k_ata_partial", "k_dlt_finish",
      "k_inl_flags", "k_inl_compact", "k_lo_prep", "k_ata_", "k_line_fit", "k_nm_")


def main():
    path = sys.argv[1]
    keys = tuple(sys.argv[2:]) or LO
    rows = list(csv.DictReader(open(path)))
    by = collections.defaultdict(list)
    for r in rows:
        by[(r["Queue_Id"], r.get("Stream_Id", ""))].append(r)
    gaps, sel_gaps, ktime, sel_ktime = [], [], 0.0, 0.0
    for q, rs in by.items():
        rs.sort(key=lambda r: int(r["Start_Timestamp"]))
        for i, r in enumerate(rs):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            ktime += e - s
            hit = any(k in r["Kernel_Name"] for k in keys)
            if hit:
                sel_ktime += e - s
            if i:
                g = s - int(rs[i - 1]["End_Timestamp"])
                if 0 <= g < 50_000:  # dependent launches (larger gaps: the host was elsewhere)
                    gaps.append(g)
                    if hit and any(k in rs[i - 1]["Kernel_Name"] for k in keys):
                        sel_gaps.append(g)
    out = {"dispatches": len(rows), "kernel_us": ktime / 1e3, "gaps_counted": len(gaps),
           "gap_median_us": statistics.median(gaps) / 1e3 if gaps else None,
           "gap_mean_us": statistics.mean(gaps) / 1e3 if gaps else None,
           "selected": {"filter": list(keys), "kernel_us": sel_ktime / 1e3, "gaps": len(sel_gaps),
                        "gap_median_us": statistics.median(sel_gaps) / 1e3 if sel_gaps else None,
                        "gap_mean_us": statistics.mean(sel_gaps) / 1e3 if sel_gaps else None,
                        "gap_total_us": sum(sel_gaps) / 1e3}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
