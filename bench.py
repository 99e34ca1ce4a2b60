#!/usr/bin/env python3
"""Hypothesis-throughput bench of the USAC hot path (BASELINE.json metric).

One step = one batch of B minimal samples on each rank: device sampler -> fused 4-pt
DLT solve -> inlier count + score of every hypothesis over all N correspondences ->
batch best (Score::bigger); with N > 1 ranks the batch bests are all-gathered over RCCL
and merged (the per-batch exchange a sharded RANSAC needs to update its termination).
Workload = BASELINE configs[1]: Homography 4-pt DLT + Uniform sampling, 10k synthetic
correspondences, 65536-hypothesis batches, 1 MI355X per rank (hypothesis-sharded:
scaling "weak", each rank owns disjoint hypothesis index ranges).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Without a launcher, --gpus N > 1 starts the N rank processes itself (launch_ranks: one per GPU,
RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, rank 0's line relayed, non-zero exit when any
rank fails); under torchrun --gpus must equal WORLD_SIZE.
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: HBM3E 8.0 TB/s


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--estimator", choices=["homography", "fundamental", "essential"], default="homography",
                    help="homography = cfg2 (the BASELINE metric's config); fundamental = cfg3; essential = cfg4 "
                         "(50k correspondences in K^-1-normalised coordinates, threshold 0.002)")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=None,
                    help="hypotheses per batch and GPU: 65536 (cfg2's stated batch; cfg4), 262144 for the cfg3 "
                         "batch-SPRT line (BASELINE configs[2] states none: at 65536 its step is the SPRT kernels' "
                         "latency, measured 0.94 vs 3.3 G hyp/s, profiles/r4c/f_sweep.txt)")
    ap.add_argument("--points", type=int, default=None, help="default: 10000 (cfg2/cfg3), 50000 (cfg4)")
    ap.add_argument("--threshold", type=float, default=None,
                    help="default: 2.0 px (cfg2/cfg3), 0.002 (cfg4, normalised coordinates)")
    ap.add_argument("--chunks", type=int, default=None, help="score point chunks (default 8 homography, 96 two-view)")
    ap.add_argument("--dlt", choices=["thin", "nullspace"], default="thin")
    ap.add_argument("--sprt", action="store_true", default=None,
                    help="batch SPRT verification (reference initial epsilon/delta for the estimator); "
                         "default on for fundamental (cfg3), off otherwise")
    ap.add_argument("--no-sprt", dest="sprt", action="store_false")
    ap.add_argument("--sampler", choices=["uniform", "prosac", "napsac"], default=None,
                    help="device sampler of the batches (default prosac for fundamental = cfg3, else uniform); "
                         "napsac = grid neighbours built on the device (cell 50), homography on the cfg5 "
                         "generator's clustered points (100k by default)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline sample (0 = skip)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cfg5", action="store_true",
                    help="BASELINE configs[4]: full USAC runs (homography + NAPSAC grid sampler + LO-RANSAC) "
                         "over 100k correspondences; one step = one run, value = main-loop hypotheses/s")
    ap.add_argument("--sprt-exact", action="store_true",
                    help="cfg3 with the reference's sequential SPRT: whole Ransac::run calls (Fundamental + PROSAC "
                         "+ SPRT, rolling pool index, adaptive history); one step = one run")
    ap.add_argument("--lo", type=int, default=1, help="cfg5 LO variant: 1 InItLORsc (unlimited), 2 InItFLORsc")
    ap.add_argument("--cfg5-replicas", action="store_true",
                    help="cfg5 with N > 1: independent runs per rank instead of hypothesis-sharded runs")
    ap.add_argument("--prewarm-ms", type=float, default=150.0,
                    help="untimed device warm-up before the warmup steps (throughput lines): batches are run "
                         "for this long first, so the timed steps see the GPU at its sustained clocks even when "
                         "--warmup is a handful of steps (0 = off)")
    ap.add_argument("--pipeline", type=int, default=None,
                    help="batches in flight: one context (stream + buffers) per in-flight batch, so batch i+1's "
                         "solve overlaps batch i's scoring (default 3; essential 16 at N = 1, else 8: its "
                         "root-order kernels are long and narrow, DESIGN.md §6)")
    args = ap.parse_args()
    ess = args.estimator == "essential"
    if args.points is None:
        args.points = 100000 if args.cfg5 or args.sampler == "napsac" else 50000 if ess else 10000
    if args.threshold is None:
        args.threshold = 0.002 if ess else 2.0
    if args.chunks is None:
        args.chunks = 8 if args.estimator == "homography" else 96
    fund = args.estimator == "fundamental"
    if args.sprt is None:
        args.sprt = fund
    if args.sampler is None:
        args.sampler = "prosac" if fund else "uniform"
    if args.batch is None:
        args.batch = 262144 if fund and args.sprt else 65536
    if args.pipeline is None:  # essential: 16 in flight at N = 1 (the N > 1 exchange ring holds 8)
        args.pipeline = (16 if args.gpus == 1 else 8) if ess else 3
    return args


def cpu_info():
    model = platform.processor() or platform.machine()
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    # the box's CPU share (OMP_NUM_THREADS is set to it there), not the whole machine
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or avail
    return model, avail, min(avail, share)


def cpu_baseline(kind, pts, thr, dlt_mode, seconds):
    """The CPU oracle's reference-style loop (glibc pool sampler, per-hypothesis minimal
    solve, full sequential score of every model), bounded samples: on one host core (the
    reference is single-threaded: the ≥10x denominator) and on all the cores the box grants
    (pthreads over disjoint hypothesis ranges, one estimator each)."""
    from oracle import oracle as O

    O.lib()
    okind = {"fundamental": O.FUNDAMENTAL, "essential": O.ESSENTIAL}.get(kind, O.HOMOGRAPHY)
    t0 = time.perf_counter()
    O.hypothesis_loop(okind, pts, thr, 1, 50, dlt_mode)
    per = max((time.perf_counter() - t0) / 50, 1e-6)
    count = max(100, int(seconds / per))
    t0 = time.perf_counter()
    O.hypothesis_loop(okind, pts, thr, 2, count, dlt_mode)
    dt = time.perf_counter() - t0
    model, avail, threads = cpu_info()
    count_mt = max(100, int(seconds / per * threads / 2))
    dt_mt, _ = O.hypothesis_loop_mt(okind, pts, thr, 3, count_mt, threads, dlt_mode)
    what = {"fundamental": "7-pt solve+oriented filter+Sampson score",
            "essential": "5-pt solve+cheirality+epipolar-distance score"}.get(kind, "DLT4+inverse+score")
    return {"value": count / dt, "unit": "hypotheses/s", "cores": 1, "kind": "port",
            "sample": "%d hypotheses of the same workload (N=%d, sample+%s, glibc sampler), %.1f s on 1 core of "
                      "%s" % (count, len(pts), what, dt, model),
            "all_cores": {"value": count_mt / dt_mt, "unit": "hypotheses/s", "cores": threads,
                          "sample": "%d hypotheses, %.1f s on %d threads" % (count_mt, dt_mt, threads)},
            "cpu_model": model, "nproc": os.cpu_count(), "cpus_available": avail}


def cpu_baseline_batch_sprt(usac, ctx, kind, pts, thr, dlt_mode, seed, first_hyp, seconds):
    """Like-for-like CPU baseline of a batch-SPRT line: the CPU oracle runs the
    SAME hypotheses the timed batches run -- the device sampler's samples at the timed indices (the
    PROSAC subset schedule, then uniform: prosac_sampler.hpp:117-172), the 7-point solve with the
    oriented-constraint filter, and the batch SPRT with the same fixed (epsilon, delta, A) from the
    same pool position per model (sprt.hpp:209-234 as a fixed walk: oracle sprt_fixed_batch) -- so its
    models per hypothesis are the GPU's by construction and its accept / reject decisions are checked
    equal.  The GPU supplies each chunk's samples and pool starts (untimed); only the oracle's solve +
    verify is timed, on one core and on the box's threads."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle as O

    okind = {"fundamental": O.FUNDAMENTAL, "essential": O.ESSENTIAL}.get(kind, O.HOMOGRAPHY)
    spk = 3 if kind == "fundamental" else 1
    m = {"fundamental": 7, "essential": 5}.get(kind, 4)
    pool, _ = O.sprt_pool(seed, okind, len(pts), m)

    def gpu_chunk(first, K):  # the device's samples, decisions and pool starts of K hypotheses
        ctx.hypothesize_async(K, seed, first, thr)
        ctx.fetch_best()
        (eps, delta, A), starts = ctx.batch_sprt_info(K * spk)
        counts, _ = ctx.last_counts(K * spk)
        return ctx.draw_samples(K, seed, first), starts, counts, (eps, delta, A)

    def cpu_chunk(ch):  # the oracle's work on one chunk: solve, oriented filter, fixed SPRT walks
        smp, starts, counts, (eps, delta, A) = ch
        est = O.Estimator(okind, pts, dlt_mode)
        om, onm = est.estimate_batch(smp)
        om = np.asarray(om, np.float32).reshape(len(smp), -1, 9)
        if spk == 3:
            occ = (np.arange(3)[None, :] < onm[:, None]).reshape(-1)
            models = om.reshape(-1, 9)[occ]
        else:
            occ = onm == 1 if okind == O.ESSENTIAL else np.ones(len(smp), bool)
            models = om[:, 0][occ]
        good, cnt, tested = O.sprt_fixed_batch(est, pool, thr, models, starts[occ], eps, delta, A)
        return int(occ.sum()), bool((cnt == counts[occ]).all()), int(good.sum()), int(tested.sum())

    # calibrate on one chunk, then a bounded sample of ~`seconds` of one core's work
    K = 8192
    c0 = gpu_chunk(first_hyp, K)
    t0 = time.perf_counter()
    cpu_chunk(c0)
    per = max((time.perf_counter() - t0) / K, 1e-7)
    nchunks = max(2, min(256, int(seconds / per / K)))
    chunks = [gpu_chunk(first_hyp + i * K, K) for i in range(nchunks)]
    t0 = time.perf_counter()
    res = [cpu_chunk(ch) for ch in chunks]
    dt = time.perf_counter() - t0
    model, avail, threads = cpu_info()
    t1 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(cpu_chunk, chunks))
    dt_mt = time.perf_counter() - t1
    hyps = nchunks * K
    models = sum(r[0] for r in res)
    return {"value": hyps / dt, "unit": "hypotheses/s", "cores": 1, "kind": "port",
            "sample": "%d hypotheses of the timed stream (device sampler indices %d..%d: the same samples), 7-pt solve "
                      "+ oriented filter + batch SPRT with the line's fixed (epsilon, delta, A) from the device's pool "
                      "starts, %.1f s on 1 core of %s" % (hyps, first_hyp, first_hyp + hyps - 1, dt, model),
            "models_per_hypothesis": models / hyps, "sprt_accepted": sum(r[2] for r in res),
            "points_tested_per_hypothesis": sum(r[3] for r in res) / hyps,
            "decisions_equal": all(r[1] for r in res),
            "all_cores": {"value": hyps / dt_mt, "unit": "hypotheses/s", "cores": threads,
                          "sample": "the same %d hypotheses, %.1f s on %d threads" % (hyps, dt_mt, threads)},
            "cpu_model": model, "nproc": os.cpu_count(), "cpus_available": avail}


def parity_check(usac, kind, pts, thr, dlt_mode, samples=None):
    """Inlier-count match vs the reference path (CPU oracle) on 256 host-drawn samples (or the
    given ones, e.g. the device NAPSAC stream's)."""
    from oracle import oracle as O

    fund = kind == "fundamental"
    ess = kind == "essential"
    m = 7 if fund else 5 if ess else 4
    if samples is None:
        samples = O.uniform_samples(77, len(pts), m, 256)
    est = O.Estimator(O.FUNDAMENTAL if fund else O.ESSENTIAL if ess else O.HOMOGRAPHY, pts, dlt_mode)
    om, onm = est.estimate_batch(samples)
    if ess:
        oc, osum = est.score_models(om, thr)
        occupied = onm == 1
        oc = np.where(occupied, oc, -1)
        osum = np.where(occupied, osum, 0).astype(np.float32)
    elif fund:
        slots = om.reshape(-1, 9)
        oc, osum = est.score_models(slots, thr)
        occupied = (np.arange(3)[None, :] < onm[:, None]).reshape(-1)
        oc = np.where(occupied, oc, -1)
        osum = np.where(occupied, osum, 0).astype(np.float32)
    else:
        oc, osum = est.score_models(om, thr)
        occupied = np.ones(len(oc), bool)
    est_id = usac.ESTIMATOR.Fundamental if fund else usac.ESTIMATOR.Essential if ess else usac.ESTIMATOR.Homography
    with usac.Context(est_id, pts, device=usac_device()) as ctx:
        ctx.set_dlt_mode(dlt_mode)
        c, s, _ = ctx.hypothesize_score(samples=samples, thr=thr)
    s = np.where(occupied, s, 0).astype(np.float32)
    return {"hypotheses": 256, "models": int(occupied.sum()), "inlier_counts_equal": bool((c == oc).all()),
            "scores_bit_equal": bool((s.view(np.int32) == osum.view(np.int32)).all())}


def timed_kernel_parity(usac, ctx, kind, pts, thr, dlt_mode, seed, sprt, first_hyp=0, xctx=None):
    """The timed configuration itself (device sampler, multi-chunk fast score kernel, batch SPRT
    when on) on one 256-sample batch against the CPU oracle on the same device-drawn samples:
    counts exact (SPRT: every accepted model's count), Σ within the throughput kernel's declared
    bound, and the batch record (Score::bigger + earliest index) against the oracle's exact
    (count, Σ).  The Σ bound per model with c inliers: two-view (exact terms, sums re-associated
    over point chunks) |Σ| c 2^-23, essential plus c thr 2^-18 (its drains' guarded residual);
    homography (stage-B terms from v_rcp / v_sqrt, DESIGN.md "Guard band": |S - 2 e| <= 2^-21 Mp
    + 2^-18 S per pair, Mp <= the dataset's max |x1|+|y1|+|x2|+|y2|) c (2^-22 Mp_max + 2^-18 thr)
    + |Σ| c 2^-23."""
    from oracle import oracle as O

    fund, ess = kind == "fundamental", kind == "essential"
    B = 256
    smp = ctx.draw_samples(B, seed, first_hyp)
    ctx.hypothesize_async(B, seed, first_hyp, thr)
    exchanged = None
    if xctx is not None:  # N > 1: this batch's record through the line's own RCCL exchange as well
        xctx.exchange_best_async(ctx, 0)
        exchanged = xctx.exchange_best_wait(0)
    rec = ctx.fetch_best()
    spk = 3 if fund else 1
    c, s = ctx.last_counts(B * spk)
    est = O.Estimator(O.FUNDAMENTAL if fund else O.ESSENTIAL if ess else O.HOMOGRAPHY, pts, dlt_mode)
    om, onm = est.estimate_batch(smp)
    if fund:
        oc, osum = est.score_models(om.reshape(-1, 9), thr)
        occ = (np.arange(3)[None, :] < onm[:, None]).reshape(-1)
    else:
        oc, osum = est.score_models(om, thr)
        occ = onm == 1 if ess else np.ones(B, bool)
    oc = np.where(occ, oc, -1)
    chk = (c >= 0) if sprt else occ
    counts_ok = bool((c[chk] == oc[chk]).all()) and (sprt or bool((c[~occ] < 0).all()))
    cnt = np.maximum(oc[chk], 0).astype(np.float64)
    ref = np.abs(osum[chk].astype(np.float64))
    bound = ref * cnt * 2.0 ** -23
    if ess:  # the guarded essential residual's terms (kernels_fund.hip essential_error_guarded)
        bound += cnt * thr * 2.0 ** -18
    if not (fund or ess):
        mp = float(np.abs(pts.astype(np.float64)).sum(1).max())
        bound += cnt * (2.0 ** -22 * mp + 2.0 ** -18 * thr)
    err = np.abs(s[chk].astype(np.float64) - osum[chk])
    if sprt:  # an accepted model's score is (float)count (sprt.hpp:276-281), not a Σ
        err, bound = np.zeros(0), np.zeros(0)
    out = {"hypotheses": B, "models": int(occ.sum()), "counts_equal": counts_ok,
           "sums_within_bound": bool((err <= bound).all()),
           "sum_max_err_over_bound": float((err / np.maximum(bound, 1e-30)).max()) if err.size else 0.0}
    if sprt:  # an accepted model scores (float)count: the record is the most inliers, earliest slot
        out["sprt_accepted"] = int((c >= 0).sum())
        best = oracle_best(np.where(c >= 0, oc, -1), np.where(c >= 0, oc, 0).astype(np.float32), c >= 0)
    else:  # the record: Score::bigger over the oracle's exact (count, Σ), earliest slot on ties
        best = oracle_best(oc, osum, occ)
    if best is not None or not sprt:
        out["best_record_equal"] = bool(best is not None and int(rec.inliers) == int(oc[best]) and
                                        int(rec.hyp_index) == first_hyp + int(best) // spk)
    out["expected_record"] = None if best is None else {"inliers": int(oc[best]),
                                                         "hyp_index": first_hyp + int(best) // spk}
    out["record"] = {"inliers": int(rec.inliers), "hyp_index": int(rec.hyp_index)}
    if exchanged is not None:  # the exchange returned this rank's own record in its slot
        out["exchanged"] = [{"inliers": int(r.inliers), "hyp_index": int(r.hyp_index)} for r in exchanged]
    out["ok"] = bool(counts_ok and out["sums_within_bound"] and out.get("best_record_equal", True))
    return out


def oracle_best(counts, sums, occupied):
    """Score::bigger (quality.hpp:22-31) over the occupied slots, earliest slot on exact ties
    (the batch argmax and usac_merge_records); None when no slot is occupied."""
    idx = np.flatnonzero(occupied)
    if not idx.size:
        return None
    c, sm = counts[idx].astype(np.int64), sums[idx].astype(np.float32)
    top = c == c.max()
    s_top = sm[top]
    return int(idx[top][int(np.flatnonzero(s_top == s_top.max())[0])])


def oracle_batch(kind, pts, thr, dlt_mode, samples):
    """The CPU oracle's models of `samples` (B x m) scored over all points: per slot (counts, Σ,
    occupied), spk slots per sample (3 for the 7-point solver's roots, else 1; counts -1 and Σ 0 on
    empty slots) -- the reference's per-hypothesis work, sample order."""
    from oracle import oracle as O

    fund, ess = kind == "fundamental", kind == "essential"
    est = O.Estimator(O.FUNDAMENTAL if fund else O.ESSENTIAL if ess else O.HOMOGRAPHY, pts, dlt_mode)
    om, onm = est.estimate_batch(samples)
    if fund:
        oc, osum = est.score_models(om.reshape(-1, 9), thr)
        occ = (np.arange(3)[None, :] < onm[:, None]).reshape(-1)
    else:
        oc, osum = est.score_models(om, thr)
        occ = onm == 1 if ess else np.ones(len(samples), bool)
    return np.where(occ, oc, -1), np.where(occ, osum, 0).astype(np.float32), occ


def oracle_batch_mt(kind, pts, thr, dlt_mode, samples, threads):
    """oracle_batch over row blocks on `threads` host threads (one oracle estimator each; ctypes
    releases the GIL), concatenated in sample order."""
    from concurrent.futures import ThreadPoolExecutor

    parts = np.array_split(np.arange(len(samples)), max(1, min(threads, len(samples))))
    with ThreadPoolExecutor(len(parts)) as ex:
        res = list(ex.map(lambda ix: oracle_batch(kind, pts, thr, dlt_mode, samples[ix]), parts))
    return tuple(np.concatenate([r[k] for r in res]) for k in range(3))


def first_batch_parity(usac, ctx, kind, pts, thr, dlt_mode, seed, B, step, world, rec, threads):
    """The first timed batch's merged record (every rank's B hypotheses, all-gathered and merged)
    against the reference's best update over the union of all ranks' samples (ransac.cpp:103-132:
    Score::bigger, the earliest hypothesis on exact ties).  Every rank's slice is keyed by (seed,
    global index), so rank 0 redraws all of them with its own device sampler and the CPU oracle
    scores them all (host threads)."""
    t0 = time.perf_counter()
    spk = 3 if kind == "fundamental" else 1
    firsts = [(step * world + r) * B for r in range(world)]
    smp = np.concatenate([ctx.draw_samples(B, seed, f) for f in firsts])
    oc, osum, occ = oracle_batch_mt(kind, pts, thr, dlt_mode, smp, threads)
    best = oracle_best(oc, osum, occ)
    exp_hyp = None if best is None else firsts[best // spk // B] + (best // spk) % B
    return {"hypotheses": int(len(smp)), "ranks": world, "models": int(occ.sum()),
            "record": {"inliers": int(rec.inliers), "hyp_index": int(rec.hyp_index)},
            "oracle_best": None if best is None else {"inliers": int(oc[best]), "hyp_index": int(exp_hyp)},
            "ok": bool(best is not None and int(rec.inliers) == int(oc[best]) and int(rec.hyp_index) == exp_hyp),
            "oracle_s": time.perf_counter() - t0,
            "note": "the merged record of the first timed batch vs Score::bigger over the oracle's exact (count, "
                    "Σ) of all %d ranks' samples, redrawn by rank 0 from (seed, global index)" % world}


def _kname_key(name):
    """(identifier, template arguments) of a kernel name as rocprofv3 writes it -- demangled
    ("void usac::k_score_hf<8, false>(...)") or, for kernels with vector-typed arguments, mangled
    ("_ZN4usac11k_score_h16ILi2ELi1ELi8EEEv...") -- so either form matches the other."""
    import re

    name = name.strip()
    m = re.match(r"_ZN4usac(\d+)", name)
    if m:
        ln, rest = int(m.group(1)), name[m.end():]
        ident, rest = rest[:ln], rest[ln:]
        args = tuple(int(v) for v in re.findall(r"L[ib](\d+)E", rest.split("EEv")[0])) if rest.startswith("I") else ()
        return ident, args
    m = re.search(r"usac::(\w+)\s*(<([^>]*)>)?", name)
    if not m:
        return name, ()
    args = ()
    if m.group(3):  # integer / bool template arguments (a type argument stays its text)
        def arg(a):
            a = a.strip()
            return 1 if a == "true" else 0 if a == "false" else int(a) if re.fullmatch(r"-?\d+", a) else a
        args = tuple(arg(a) for a in m.group(3).split(","))
    return m.group(1), args


def _profile_entry(kernel_prefix, n_points, batch):
    """(summary entry, source) of `kernel_prefix` in the newest committed rocprofv3 summary
    (profiles/<round>_summary.json, made by tools/archive/profile.sh + tools/summarize_profile.py)
    that ran the same workload shape; else None."""
    import glob

    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_summary.json"))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        shape = d.get("workload", {})  # only summaries of the same workload shape count
        if shape.get("n_points") != n_points or shape.get("batch") != batch:
            continue
        for k, v in d.get("kernels", {}).items():
            if k.replace(" ", "").startswith(kernel_prefix.replace(" ", "")) or _kname_key(k) == _kname_key(kernel_prefix):
                best = (v, os.path.relpath(f, ROOT))
    return best


# VALU issue peak: 1024 SIMDs (256 CUs x 4), each issuing one wave64 VALU instruction per 2
# cycles at 2.4 GHz (MI355X_MICROARCH.md, wave scheduling); a v_pk_fma_f32 occupies two such
# slots (tools/ubench/valu_rate.hip), which SQ_ACTIVE_INST_VALU (VALU-busy quad-cycles per
# wave, summed over waves) accounts for and SQ_INSTS_VALU (instructions) does not.
SIMD_CYCLES_S = 1024 * 2.4e9
VALU_PEAK_INSTR_S = SIMD_CYCLES_S / 2
MFMA_F16_DENSE_TFLOPS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense BF16/FP16


def valu_roofline(kernel_prefix, n_points, batch, kernel_ms):
    """Primary roofline of the score kernel (it is fp32-VALU-issue bound, its point
    set L2-resident): VALU-busy SIMD-cycles per launch (SQ_ACTIVE_INST_VALU x 4, committed PMC
    summary of the same workload) / this run's measured kernel time, against 1024 SIMDs x
    2.4 GHz.  Beside it: the instruction-count form (SQ_INSTS_VALU vs one wave64 instruction per
    2 cycles, packed FMAs counted once), VALUBusy straight from the PMC pass (clock-free), the
    wave-cycle split and the counter-measured HBM traffic."""
    e = _profile_entry(kernel_prefix, n_points, batch)
    if e is None or not kernel_ms:
        return None
    pmc, src = e[0].get("pmc", {}), e[1]
    t = kernel_ms * 1e-3
    out = {"bound": "valu", "unit": "SIMD-cycles/s", "peak": SIMD_CYCLES_S, "source": src}
    act = pmc.get("SQ_ACTIVE_INST_VALU")
    if act:
        out["achieved"] = act * 4 / t
        out["frac"] = out["achieved"] / SIMD_CYCLES_S
        out["valu_busy_cycles_per_launch"] = act * 4
        if pmc.get("GRBM_GUI_ACTIVE"):  # GRBM_GUI_ACTIVE is summed over the 8 XCDs (18.9 "GHz" per ns)
            out["valu_busy_pmc"] = act * 4 / 1024 / (pmc["GRBM_GUI_ACTIVE"] / 8)
    n_instr = pmc.get("SQ_INSTS_VALU")
    if n_instr:
        out["instructions_per_launch"] = n_instr
        out["instr_issue_frac"] = n_instr / t / VALU_PEAK_INSTR_S
        # issue costs over the hot loop's instruction mix from the ISA (tools/isa_mix.py): the per-
        # opcode costs measured on an MI355X (profiles/r4/valu_issue_costs.json, 8 waves per SIMD:
        # v_fma/add/mul_f32 with VGPR operands ~2.4 SIMD cycles, v_pk_fma_f32 ~4.3, v_max / v_cmp /
        # |.|-modified or SGPR-sourced plain ops ~3.9-4.3) give frac; frac_guide prices the same mix
        # at the guide's 2 (plain) / 4 (packed, transcendental); frac_x4 = SQ_ACTIVE_INST_VALU x 4,
        # which charges every instruction 4 (the counter counts ~1 per instruction, packed or not)
        import re
        mixn = "isa_%s.json" % re.sub(r"[^A-Za-z0-9]+", "_", kernel_prefix.replace("void usac::", "")).strip("_")
        mixf = os.path.join(ROOT, "profiles", "r5", mixn)
        if not os.path.exists(mixf):
            mixf = os.path.join(ROOT, "profiles", "r4", mixn)
        if os.path.exists(mixf):
            mx = json.load(open(mixf))
            guide = float(mx["issue_cycles_per_valu_instruction"])
            cyc = float(mx.get("measured_cycles_per_valu_instruction", guide))
            out["frac_x4"] = out.get("frac")
            out["frac_guide"] = n_instr * guide / t / SIMD_CYCLES_S
            out["achieved"] = n_instr * cyc / t
            out["frac"] = out["achieved"] / SIMD_CYCLES_S
            out["issue_model"] = {"cycles_per_valu_instruction": cyc, "guide_cycles_per_valu_instruction": guide,
                                  "loop_mix": mx["mix"], "by_opcode": mx.get("measured_by_opcode"),
                                  "source": os.path.relpath(mixf, ROOT), "costs": mx.get("measured_source"),
                                  "note": "frac = SQ_INSTS_VALU x the hot loop's mean measured issue cycles / kernel "
                                          "time / (1024 SIMDs x 2.4 GHz); frac_guide = the same with the guide's "
                                          "2 / 4 cycles; frac_x4 = the SQ_ACTIVE_INST_VALU x 4 form"}
    if "k_score_h16" in kernel_prefix:  # the matrix-core prefilter: its MFMA work beside the VALU issue
        # executed v_mfma_f32_32x32x16_f16 flops per launch: ceil(B / 20) waves (2 tiles of 10 hypotheses)
        # x ceil(N / 32) point blocks x 2 MFMAs x 32 x 32 x 16 x 2
        fl = -(-batch // 20) * -(-n_points // 32) * 2 * 32 * 32 * 16 * 2
        out["mfma"] = {"executed_flops_per_launch": fl, "achieved_tflops": fl / t / 1e12,
                       "peak_tflops": MFMA_F16_DENSE_TFLOPS, "frac": fl / t / 1e12 / MFMA_F16_DENSE_TFLOPS,
                       "note": "dense fp16 MFMA peak (MI355X_MICROARCH.md: ~2.5 PF); the tiles carry 9 of 16 K "
                               "columns and 30 of 32 rows, so useful flops are 0.53x the executed ones"}
        if pmc.get("SQ_VALU_MFMA_BUSY_CYCLES"):
            out["mfma"]["busy_frac_pmc"] = pmc["SQ_VALU_MFMA_BUSY_CYCLES"] / t / SIMD_CYCLES_S
    if pmc.get("SQ_WAVE_CYCLES"):
        wc = pmc["SQ_WAVE_CYCLES"]
        out["wave_cycle_split"] = {k.lower(): pmc[k] / wc for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                                    "SQ_ACTIVE_INST_ANY") if k in pmc}
    if "hbm_bytes_per_launch" in e[0]:
        hb = e[0]["hbm_bytes_per_launch"]
        out["hbm"] = {"traffic_bytes_per_launch": hb, "achieved_gbs": hb / t / 1e9, "peak_gbs": HBM_PEAK_GBS,
                      "frac": hb / t / 1e9 / HBM_PEAK_GBS}
    return out


def _stage_kernels(estimator, sprt, chunks, stage):
    """The kernels of one timed stage of a batch (usac_hypothesize_async: solve = ev0..ev1,
    score = ev1..ev2), as rocprofv3 names them (prefixes, spaces ignored)."""
    est = {"fundamental": 3, "essential": 4}.get(estimator, 2)
    if stage == "solve":
        return {2: ["usac::k_solve_h4("], 3: ["usac::k_solve_f7("],
                4: ["usac::k_e5_basis(", "usac::k_e5_dets(", "usac::k_e5_roots(", "usac::k_e5_null(",
                    "usac::k_e5_check(", "usac::k_e5_select(", "usac::k_e5_order(", "usac::k_e5_order_tail("]}[est]
    if sprt:
        return ["void usac::k_sprt_head<%d>(" % est, "void usac::k_sprt_tail<%d>(" % est]
    if est == 2:  # the matrix-core prefilter scorer (kernels_h16.hip; USAC_H16=0: k_presort_h + k_score_hf)
        if os.environ.get("USAC_H16", "1") == "0":
            return ["usac::k_presort_h(", "void usac::k_score_hf<%d, false>(" % chunks]
        ks = ["void usac::k_score_h16<2, 1, 8>("]
        if os.environ.get("USAC_H16_FUSE", "1") == "0":  # the rows by their own kernel, not the solver
            ks = ["usac::k_h16_rows("] + ks
        if os.environ.get("USAC_H16_DEFER", "1") == "0":  # the chunk sums by their own kernel, not the argmax
            ks = ks + ["usac::k_h16_finish("]
        return ks
    if est == 4 and os.environ.get("USAC_E16", "1") != "0":  # the matrix-core prefilter scorer (kernels_e16.hip)
        return ["usac::k_e16_rows(", "usac::k_score_e16(", "usac::k_e16_finish("]
    return ["usac::k_prepare_rec(", "void usac::k_presort_tv<%d>(" % est, "void usac::k_score_f2<%d>(" % est,
            "usac::k_tv_combine("]


def stage_roofline(prefixes, n_points, batch, stage_ms):
    """VALU roofline of a stage of kernels: the VALU-busy SIMD-cycles of all its kernels per
    batch (PMC SQ_ACTIVE_INST_VALU x 4, committed summary of the same workload shape) over the
    stage's time measured live with HIP events on the context stream, against 1024 SIMDs x
    2.4 GHz; per kernel, the same fraction against its own rocprofv3 duration, the wave-cycle
    split and the counter-measured HBM bytes.  None without a summary for every kernel."""
    ents = [(p, _profile_entry(p, n_points, batch)) for p in prefixes]
    if any(e is None or "SQ_ACTIVE_INST_VALU" not in e[0].get("pmc", {}) for _, e in ents):
        return None
    if not stage_ms:  # no live stage time: the kernels' own rocprofv3 durations, back to back
        stage_ms = sum(e[0].get("trace", {}).get("avg_ns", 0.0) for _, e in ents) * 1e-6
        if not stage_ms:
            return None
    t = stage_ms * 1e-3
    busy = sum(e[0]["pmc"]["SQ_ACTIVE_INST_VALU"] * 4 for _, e in ents)
    hbm = sum(e[0].get("hbm_bytes_per_launch", 0.0) for _, e in ents)
    out = {"bound": "valu", "unit": "SIMD-cycles/s", "peak": SIMD_CYCLES_S, "achieved": busy / t,
           "frac": busy / t / SIMD_CYCLES_S, "valu_busy_cycles_per_launch": busy, "stage_ms": stage_ms,
           "sources": sorted({e[1] for _, e in ents}),
           "hbm": {"traffic_bytes_per_launch": hbm, "achieved_gbs": hbm / t / 1e9, "peak_gbs": HBM_PEAK_GBS,
                   "frac": hbm / t / 1e9 / HBM_PEAK_GBS}, "kernels": {}}
    for p, (v, _) in ents:
        pmc = v["pmc"]
        k = {"rocprof_avg_us": v.get("trace", {}).get("avg_ns", 0.0) / 1e3,
             "valu_busy_cycles": pmc["SQ_ACTIVE_INST_VALU"] * 4}
        if k["rocprof_avg_us"]:
            k["valu_frac"] = k["valu_busy_cycles"] / (k["rocprof_avg_us"] * 1e-6) / SIMD_CYCLES_S
        if pmc.get("SQ_WAVE_CYCLES"):
            k["wave_cycle_split"] = {c.lower(): pmc[c] / pmc["SQ_WAVE_CYCLES"]
                                     for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY") if c in pmc}
        if "hbm_bytes_per_launch" in v:
            k["hbm_bytes"] = v["hbm_bytes_per_launch"]
        out["kernels"][p.replace("void ", "").replace("usac::", "").rstrip("(")] = k
    return out


def run_roofline(n_points, run_ms):
    """Roofline of a full-run workload (cfg5) from the committed rocprofv3 summary of its own runs
    (profiles/r*_summary.json with workload batch 0 and the number of runs profiled: every dispatch
    counted, tools/profile_round.sh cfg5).  Per kernel: calls per run, average duration, device time
    per run and VALU-busy SIMD-cycles per dispatch (PMC SQ_ACTIVE_INST_VALU x 4).  The dominant
    kernel -- most device time per run -- is priced against the VALU issue peak over its own
    average duration (and its counter-measured HBM bytes against HBM peak); beside it the share of
    the run's wall time the device spends in kernels at all (the rest is host replay and launch
    latency of the run's dependent steps)."""
    import glob

    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_summary.json"))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        w = d.get("workload", {})
        if w.get("n_points") == n_points and w.get("batch") == 0 and w.get("runs"):
            best = (d, os.path.relpath(f, ROOT))
    if best is None:
        return None
    d, src = best
    runs = d["workload"]["runs"]
    rows = []
    for k, v in d["kernels"].items():
        tr = v.get("trace")
        if not tr or not tr.get("avg_ns"):
            continue
        pmc = v.get("pmc", {})
        r = {"kernel": k.split("(")[0].replace("void ", "").replace("usac::", ""), "calls_per_run": tr["calls"] / runs,
             "avg_us": tr["avg_ns"] / 1e3, "device_us_per_run": tr["calls"] / runs * tr["avg_ns"] / 1e3}
        if pmc.get("SQ_ACTIVE_INST_VALU"):
            r["valu_frac"] = pmc["SQ_ACTIVE_INST_VALU"] * 4 / (tr["avg_ns"] * 1e-9) / SIMD_CYCLES_S
        if "hbm_bytes_per_launch" in v:
            r["hbm_bytes"] = v["hbm_bytes_per_launch"]
            r["hbm_frac"] = v["hbm_bytes_per_launch"] / (tr["avg_ns"] * 1e-9) / 1e9 / HBM_PEAK_GBS
        rows.append(r)
    if not rows:
        return None
    rows.sort(key=lambda r: -r["device_us_per_run"])
    top = rows[0]
    dev_us = sum(r["device_us_per_run"] for r in rows)
    t = top["avg_us"] * 1e-6
    busy = top.get("valu_frac", 0.0) * t * SIMD_CYCLES_S
    return {"bound": "valu", "unit": "SIMD-cycles/s", "peak": SIMD_CYCLES_S, "achieved": busy / t,
            "frac": top.get("valu_frac"), "kernel": top["kernel"], "kernel_avg_us": top["avg_us"],
            "traffic": top.get("hbm_bytes"), "traffic_unit": "bytes/launch",
            "hbm": {"achieved_gbs": (top.get("hbm_bytes") or 0.0) / t / 1e9, "peak_gbs": HBM_PEAK_GBS,
                    "frac": top.get("hbm_frac")},
            "source": src, "runs_profiled": runs,
            "device_us_per_run": dev_us, "run_ms": run_ms,
            "device_busy_frac_of_run": dev_us * 1e-3 / run_ms if run_ms else None,
            "kernels_by_device_time": rows[:12],
            "note": "the kernels the cfg5 runs execute (trace of bench.py --cfg5 itself): the dominant one by "
                    "device time per run, VALU-busy cycles per dispatch / its average duration / (1024 SIMDs x "
                    "2.4 GHz); device_busy_frac_of_run = summed kernel time per run / this line's ms per run"}


_DEV = 0


def usac_device():
    return _DEV


def cfg5_main(args, usac, synthetic, dist, torch, world, rank, local_rank):
    """Full-run mode (BASELINE configs[4]): whole USAC loops -- batched device solve + score of
    the NAPSAC samples, exact host replay of the sequential loop, LO-RANSAC (every LSQ fit and
    inlier scan on the device).  With N > 1 ranks each run is hypothesis-sharded (SURVEY §8(e),
    usac_ransac_run_sharded: every batch split over the ranks, counts and models all-gathered
    over RCCL, the replay identical on every rank) -- strong scaling, value = main-loop
    hypotheses of the runs / max wall time; --cfg5-replicas runs independent seeds per rank
    instead (weak scaling, value summed over ranks)."""
    from oracle import oracle as O

    pts, _, _ = synthetic.homography_points(n=args.points, inlier_ratio=0.2, seed=args.seed, cluster=(500, 500, 150))
    max_iters = 5000

    def model(seed):
        mdl = usac.Model(args.threshold, 4, 0.95, 7, usac.ESTIMATOR.Homography, usac.SAMPLER.Napsac)
        mdl.ResetRandomGenerator(False)
        mdl.setSeed(seed)
        mdl.lo = usac.LocOpt(args.lo)
        mdl.max_iterations = max_iters
        mdl.setNeighborsType(usac.NeighborsSearch.Grid)
        return mdl

    sharded = world > 1 and not args.cfg5_replicas
    comm_ctx, rccl = None, None
    if sharded:  # the RCCL communicator lives on one context; each run's context borrows it via the bench
        comm_ctx = usac.Context(usac.ESTIMATOR.Homography, pts, device=local_rank)
        uid = [usac.Context.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        exchange = init_exchange(comm_ctx, usac, dist, torch, world, rank, uid[0])
        rccl = rccl_report(comm_ctx, exchange, dist, world, rank)

    def gloo_gather(b):
        t = torch.frombuffer(bytearray(b), dtype=torch.uint8)
        parts = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        return [p.numpy().tobytes() for p in parts]

    # replicas: one context per rank on its own device, runs back to back on it (the points stay
    # in HBM and the context's device NAPSAC grid is built once per cell size)
    run_ctx = None if sharded else usac.Context(usac.ESTIMATOR.Homography, pts, device=local_rank)

    def one_run(seed):
        if not sharded:
            r = usac.Ransac(model(seed), pts, ctx=run_ctx)
            r.run()
            return r.getRansacOutput()
        r = usac.Ransac(model(seed), pts, ctx=comm_ctx)
        r.run(shard=(world, rank, "rccl" if exchange == "rccl_allgather" else gloo_gather))
        return r.getRansacOutput()

    for i in range(args.warmup):
        one_run(10_000 + i)
    if world > 1:
        dist.barrier()
    iters = 0
    t0 = time.perf_counter()
    for step in range(args.steps):
        seed = args.seed + step if sharded else args.seed + step * world + rank
        iters += one_run(seed).getNumberOfMainIterations()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed, float(iters)], dtype=torch.float64)
        dist.all_reduce(tt[:1], op=dist.ReduceOp.MAX)
        if not sharded:  # replicas: every rank's runs are distinct work
            dist.all_reduce(tt[1:], op=dist.ReduceOp.SUM)
        elapsed, iters = float(tt[0]), int(tt[1])
    # parity: one run against the oracle (same seed) -- every rank takes part in a sharded run
    out = one_run(args.seed)
    if rank != 0:
        return
    n = args.points
    run_ms = elapsed / args.steps * 1e3
    # parity of that run: iterations, LO counters, model, inliers
    ref = O.ransac_run(O.HOMOGRAPHY, pts, args.threshold, 0.95, args.seed, sampler=O.SAMPLER_NAPSAC, sprt=False,
                       lo=args.lo, max_iters=max_iters)
    # the kernels these runs execute, from the committed trace + PMC summary of this same command
    # (tools/profile_round.sh cfg5: every dispatch of its runs)
    roof = run_roofline(n, run_ms) or {
        "bound": "valu", "achieved": None, "peak": SIMD_CYCLES_S, "unit": "SIMD-cycles/s", "frac": None,
        "traffic": None, "note": "no committed cfg5 summary (profiles/r*_summary.json, workload batch 0)"}
    parity = {"runs": 1, "iterations_equal": out.getNumberOfMainIterations() == ref["iters"],
              "lo_iters_equal": out.getLOIters() == ref["lo_inner_iters"],
              "model_bit_equal": bool((np.asarray(out.getModel(), np.float32).view(np.int32) ==
                                       np.asarray(ref["model"], np.float32).view(np.int32)).all()),
              "inliers_equal": bool(np.array_equal(out.getInliers(), ref["inlier_idx"]))}
    line = {
        "metric": "model hypotheses/sec (sample+solve+score) and inlier-count match vs ref",
        "value": iters / elapsed, "unit": "hypotheses/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "strong" if sharded else "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (clustered homography inliers 20%%, uniform outliers), %d correspondences" % n,
        "config": {"workload": "cfg5: Homography_estimator + Napsac_sampler (grid) + LO-RANSAC (%s), full runs, "
                               "%d correspondences; one step = one run per rank" %
                               ("InItLORsc" if args.lo == 1 else "InItFLORsc", n),
                   "n_points": n, "threshold": args.threshold, "max_iterations": max_iters,
                   "hypotheses_per_gpu": iters / world,
                   "parallelism": ("hypothesis-sharded runs x%d (%s)" % (world, exchange)) if sharded else
                                  "replicas x%d" % world, "rccl": rccl},
        "roofline": roof,
        "parity": parity,
        "run_stats": {k: int(out.raw[k]) for k in ("batches", "n_records", "lo_rounds", "lo_stages", "sum_models",
                                                     "lo_iterative_iters", "polish_passes")},
    }
    line["run_stats"]["lo_inner_iters"] = int(out.getLOIters())
    line["run_stats"]["time_us"] = int(out.getTimeMicroSeconds())
    if args.cpu_seconds > 0:
        t1 = time.perf_counter()
        runs, it = 0, 0
        while runs == 0 or time.perf_counter() - t1 < args.cpu_seconds:
            r = O.ransac_run(O.HOMOGRAPHY, pts, args.threshold, 0.95, args.seed + 1000 + runs, sampler=O.SAMPLER_NAPSAC,
                             sprt=False, lo=args.lo, max_iters=max_iters)
            it += r["iters"]
            runs += 1
        dt = time.perf_counter() - t1
        model_name, avail, threads = cpu_info()

        def worker(k):  # full oracle runs until the deadline (ctypes releases the GIL; the oracle is reentrant)
            w_it, w_runs, end = 0, 0, time.perf_counter() + args.cpu_seconds / 2
            while w_runs == 0 or time.perf_counter() < end:
                r = O.ransac_run(O.HOMOGRAPHY, pts, args.threshold, 0.95, args.seed + 100000 * (k + 1) + w_runs,
                                 sampler=O.SAMPLER_NAPSAC, sprt=False, lo=args.lo, max_iters=max_iters)
                w_it += r["iters"]
                w_runs += 1
            return w_it, w_runs

        from concurrent.futures import ThreadPoolExecutor
        t2 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            res = list(ex.map(worker, range(threads)))
        dt_mt = time.perf_counter() - t2
        it_mt, runs_mt = sum(r[0] for r in res), sum(r[1] for r in res)
        line["cpu_baseline"] = {"value": it / dt, "unit": "hypotheses/s", "cores": 1, "kind": "port",
                                "sample": "%d full runs (%d hypotheses, NAPSAC + LO, N=%d), %.1f s on 1 core of %s" %
                                          (runs, it, n, dt, model_name),
                                "all_cores": {"value": it_mt / dt_mt, "unit": "hypotheses/s", "cores": threads,
                                              "sample": "%d full runs (%d hypotheses), %.1f s on %d threads" %
                                                        (runs_mt, it_mt, dt_mt, threads)},
                                "cpu_model": model_name, "nproc": os.cpu_count(), "cpus_available": avail}
    print(json.dumps(line))


def cfg3_exact_main(args, usac, synthetic, dist, torch, world, rank, local_rank):
    """cfg3 with the reference's own SPRT (--sprt-exact): whole Ransac::run calls (BASELINE
    configs[2]: Fundamental 7-pt + PROSAC + SPRT, 10 k quality-sorted correspondences) through
    usac_ransac_run, whose SPRT is the reference's sequential fp64 lambda walk over the rolling pool
    index with the adaptive history (sprt.hpp:191-317, on device-computed pool-order inlier words).
    One step = one run per rank (seeds differ), value = main-loop hypotheses (SPRT double counting
    included, ransac.cpp:81-83) / wall time; N > 1: replicas (weak scaling).  Parity: runs compared
    with the oracle -- iterations, records, SPRT rejections and history length, PROSAC termination
    length, model bits, inlier list."""
    from oracle import oracle as O

    n = args.points
    pts, _, _ = synthetic.fundamental_points(n=n, inlier_ratio=0.3, seed=args.seed)  # quality-sorted (PROSAC)

    mdl = usac.Model(args.threshold, 7, 0.95, 7, usac.ESTIMATOR.Fundamental, usac.SAMPLER.Prosac)
    mdl.ResetRandomGenerator(False)
    mdl.setSprt(True)

    def model(seed):  # one parameter object, re-seeded per run (usac.Model.setSeed)
        mdl.setSeed(seed)
        return mdl

    ctx = usac.Context(usac.ESTIMATOR.Fundamental, pts, device=local_rank)  # one context, runs back to back

    def one_run(seed):
        r = usac.Ransac(model(seed), pts, ctx=ctx)
        r.run()
        return r

    for i in range(args.warmup):
        one_run(10_000 + i)
    if world > 1:
        dist.barrier()
    iters, rejected, batches, lib_us, rewinds = 0, 0, 0, 0, 0
    t0 = time.perf_counter()
    for step in range(args.steps):
        r = one_run(args.seed + step * world + rank)
        out = r.getRansacOutput()
        iters += out.getNumberOfMainIterations()
        rejected += out.raw["sprt_rejected"]
        batches += out.raw["batches"]
        rewinds += out.raw["rollbacks"]
        lib_us += out.getTimeMicroSeconds()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed, float(iters)], dtype=torch.float64)
        dist.all_reduce(tt[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(tt[1:], op=dist.ReduceOp.SUM)
        elapsed, iters = float(tt[0]), int(tt[1])
    if rank != 0:
        ctx.close()
        return
    # parity: the first runs of the timed seeds against the oracle
    checks = []
    for k in range(min(args.steps, 8)):
        seed = args.seed + k * world
        r = one_run(seed)
        out = r.getRansacOutput()
        ref = O.ransac_run(O.FUNDAMENTAL, pts, args.threshold, 0.95, seed, sampler=O.SAMPLER_PROSAC, sprt=True)
        checks.append({
            "iterations_equal": out.getNumberOfMainIterations() == ref["iters"],
            "records_equal": [(i, c, float(np.float32(s))) for i, c, s in r.records] ==
                             [(i, c, float(np.float32(s))) for i, c, s in ref["records"]],
            "sprt_rejected_equal": out.raw["sprt_rejected"] == ref["sprt_rejected"],
            "sprt_histories_equal": out.raw["sprt_histories"] == ref["sprt_histories"],
            "prosac_term_len_equal": out.raw["prosac_term_len"] == ref["prosac_term_len"],
            "model_bit_equal": bool((np.asarray(out.getModel(), np.float32).view(np.int32) ==
                                     np.asarray(ref["model"], np.float32).view(np.int32)).all()),
            "inliers_equal": bool(np.array_equal(out.getInliers(), ref["inlier_idx"]))})
    parity = {"runs": len(checks)}
    for key in checks[0]:
        parity[key] = all(c[key] for c in checks)
    # roofline of the run's dominant kernel: the SPRT pool-order inlier words of one batch
    roof = stage_roofline(["void usac::k_pool_mask<3>(", "usac::k_solve_f7("], n, 1024, None) or {
        "bound": "valu", "achieved": None, "peak": SIMD_CYCLES_S, "unit": "SIMD-cycles/s", "frac": None}
    roof.update({"traffic": roof.get("hbm", {}).get("traffic_bytes_per_launch"),
                 "note": "a run is the host's sequential SPRT walk over device-computed pool-order inlier words "
                         "(k_pool_mask) of batches of 1024 PROSAC samples (k_solve_f7), with host round trips per "
                         "batch; see DESIGN.md §7 (cfg3 exact line) for the per-run split"})
    line = {
        "metric": "model hypotheses/sec (sample+solve+score) and inlier-count match vs ref",
        "value": iters / elapsed, "unit": "hypotheses/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (SURVEY §8(d) cfg3 generator: two views, 30% inliers, 0.5 px noise, quality-sorted)",
        "config": {"workload": "cfg3 exact: Fundamental_estimator (7-pt) + Prosac_sampler + the reference's sequential "
                               "SPRT (rolling pool index, adaptive history, fp64 lambda), full Ransac::run calls, "
                               "%d correspondences; one step = one run per rank" % n,
                   "n_points": n, "threshold": args.threshold, "sprt": "exact sequential (sprt.hpp:191-317)",
                   "hypotheses_per_gpu": iters / world, "parallelism": "replicas x%d" % world},
        "roofline": roof,
        "parity": parity,
        "run_stats": {"iterations_per_run": iters / world / args.steps, "sprt_rejected": rejected,
                      "batches": batches,
                      # PROSAC redraws: a best update that shrinks the termination length below a
                      # later sample's subset cuts the batch there (a new device batch follows)
                      "prosac_rewinds": rewinds,
                      # rank 0's usac_ransac_run wall time per run (RansacOutput.getTimeMicroSeconds:
                      # argument checks to the polish's end) beside the line's per-run wall time
                      "library_ms_per_run": lib_us / 1e3 / args.steps},
    }
    if args.cpu_seconds > 0:
        t1 = time.perf_counter()
        runs, it = 0, 0
        while runs == 0 or time.perf_counter() - t1 < args.cpu_seconds:
            r = O.ransac_run(O.FUNDAMENTAL, pts, args.threshold, 0.95, args.seed + 1000 + runs,
                             sampler=O.SAMPLER_PROSAC, sprt=True)
            it += r["iters"]
            runs += 1
        dt = time.perf_counter() - t1
        model_name, avail, _ = cpu_info()
        line["cpu_baseline"] = {"value": it / dt, "unit": "hypotheses/s", "cores": 1, "kind": "port",
                                "sample": "%d full runs (%d hypotheses, PROSAC + SPRT, N=%d), %.1f s on 1 core of %s"
                                          % (runs, it, n, dt, model_name)}
        line["gpu_over_cpu"] = line["value"] / line["cpu_baseline"]["value"]
    ctx.close()
    print(json.dumps(line))


def init_exchange(ctx, usac, dist, torch, world, rank, uid):
    """RCCL communicator for the per-batch record exchange.  Ranks on distinct GPUs must get
    one: a failure ends the run (exit 3) instead of reporting a scaling line without RCCL.
    Only the USAC_BENCH_SAME_DEVICE rehearsal (several ranks on one GPU, which RCCL refuses)
    falls back to exchanging the 56-byte records over gloo."""
    try:
        ctx.comm_init(world, rank, uid)
        ok = 1
    except usac.UsacError as e:
        print("bench: RCCL init failed on rank %d (%s)" % (rank, e), file=sys.stderr)
        ok = 0
    t = torch.tensor([ok])
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    if int(t) == 1:
        return "rccl_allgather"
    if os.environ.get("USAC_BENCH_SAME_DEVICE"):
        return "gloo_allgather"
    print("bench: no RCCL communicator on distinct devices; refusing to report a scaling line", file=sys.stderr)
    sys.exit(3)


def rccl_report(ctx, exchange, dist, world, rank):
    """The rank count RCCL itself reports for the line's communicator (ncclCommCount /
    ncclCommUserRank / ncclCommCuDevice through usac_comm_count), gathered from every rank; a line
    whose communicator does not hold N ranks, or whose ranks do not sit on N distinct devices, is
    refused (exit 4).  None without an RCCL exchange (N = 1, or the one-GPU gloo rehearsal)."""
    if exchange != "rccl_allgather":
        return None
    n, r, dev = ctx.comm_count()
    allv = [None] * world
    dist.all_gather_object(allv, (n, r, dev))
    bad = [v for k, v in enumerate(allv) if v[0] != world or v[1] != k]
    if bad or len({v[2] for v in allv}) != world:
        if rank == 0:
            print("bench: RCCL reports %r for %d ranks; refusing to report the line" % (allv, world), file=sys.stderr)
        sys.exit(4)
    return {"ranks": n, "devices": [v[2] for v in allv], "source": "ncclCommCount / ncclCommUserRank / "
                                                                     "ncclCommCuDevice"}


def ranks_parity(usac, tk_all, exchange):
    """N > 1: every rank's 256-sample timed-configuration check (counts exact, Σ within bound,
    local record = the oracle's best), the merge of the ranks' records (usac_merge_records) equal
    to Score::bigger over the ranks' oracle-expected records (ransac.cpp:103-132; earliest
    hypothesis on ties), and -- with RCCL -- the exchange's all-gathered list equal to the records
    the ranks hold."""
    recs = [t["record"] for t in tk_all]
    exp = [t["expected_record"] for t in tk_all]
    merged = usac.merge_records([usac.Record(hyp_index=r["hyp_index"], inliers=r["inliers"],
                                             score=float(r["inliers"]), valid=1) for r in recs]) \
        if all(t.get("sprt_accepted") is not None for t in tk_all) else None
    # the expected merge: the most inliers, then the earliest hypothesis (the slices are disjoint and
    # ascending in rank order; with equal counts across ranks the exact Σ decides, which only the
    # SPRT lines -- score = count -- leave to the index)
    cand = [e for e in exp if e is not None]
    out = {"per_rank_ok": [bool(t["ok"]) for t in tk_all], "records": recs}
    if cand and merged is not None:
        top = max(e["inliers"] for e in cand)
        want = min((e for e in cand if e["inliers"] == top), key=lambda e: e["hyp_index"])
        out["expected_merge"] = want
        out["merge_equal"] = int(merged.inliers) == want["inliers"] and int(merged.hyp_index) == want["hyp_index"]
    if exchange == "rccl_allgather":
        out["exchange_equal"] = all(t.get("exchanged") == recs for t in tk_all)
    out["ok"] = bool(all(out["per_rank_ok"]) and out.get("merge_equal", True) and out.get("exchange_equal", True))
    return out


def launch_plan(gpus, env):
    """How `bench.py --gpus N` runs, decided before anything touches the GPU:
    ("self", 1) -- one process, one GPU (no WORLD_SIZE, N = 1);
    ("rank", W) -- this process is one rank of a launcher's W (torchrun, or launch_ranks below);
    ("spawn", N) -- no launcher: start N rank processes here (launch_ranks);
    ("refuse", msg) -- --gpus disagrees with the launcher's WORLD_SIZE."""
    if gpus < 1:
        return "refuse", "--gpus must be >= 1"
    ws = env.get("WORLD_SIZE")
    if ws is None or ws == "":
        return ("spawn", gpus) if gpus > 1 else ("self", 1)
    try:
        world = int(ws)
    except ValueError:
        return "refuse", "WORLD_SIZE=%r is not an integer" % ws
    if world != gpus:
        return "refuse", "--gpus %d but the launcher's WORLD_SIZE is %d: refusing to report a %d-GPU line" % (
            gpus, world, gpus)
    return "rank", world


def _free_port():
    import socket

    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv, env=None, script=None):
    """One process per GPU without torchrun: N fresh children of this (GPU-untouched) parent, each
    with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT, running this script
    with the same arguments.  Rank 0's stdout (the JSON line) is relayed; the other ranks' stdout
    goes to stderr.  When a child fails the others are ended (they would wait in a collective) and
    the launcher exits with the failing child's status; 0 only when every rank exits 0."""
    import subprocess
    import threading

    base = dict(os.environ if env is None else env)
    base.update({"WORLD_SIZE": str(n), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(_free_port()),
                 "LOCAL_WORLD_SIZE": str(n)})
    procs = []
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, "-u", script or os.path.abspath(__file__)] + list(argv),
                                      env=e, stdout=subprocess.PIPE, text=True))

    def relay(p, out):
        for ln in p.stdout:
            out.write(ln)
            out.flush()
    th = [threading.Thread(target=relay, args=(p, sys.stdout if r == 0 else sys.stderr), daemon=True)
          for r, p in enumerate(procs)]
    for t in th:
        t.start()
    status = 0
    while True:
        codes = [p.poll() for p in procs]
        failed = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if failed and status == 0:
            r, status = failed[0]
            print("bench: rank %d exited with status %d; ending the other ranks" % (r, status), file=sys.stderr)
            for p in procs:
                if p.poll() is None:
                    p.terminate()
        if all(c is not None for c in codes):
            break
        time.sleep(0.05)
    for t in th:
        t.join(timeout=5)
    return status


def main():
    global _DEV
    args = parse()
    how, what = launch_plan(args.gpus, os.environ)
    if how == "refuse":
        print("bench: " + what, file=sys.stderr)
        sys.exit(2)
    if how == "spawn":  # no HIP call has happened in this process
        sys.exit(launch_ranks(what, sys.argv[1:]))
    if os.environ.get("USAC_BENCH_DRY_RUN"):  # launcher plumbing test: report the rank's view and stop
        r = int(os.environ.get("RANK", "0"))
        if os.environ.get("USAC_BENCH_FAIL_RANK") == str(r):
            sys.exit(5)
        if r == 0:
            print(json.dumps({"n_gpus": what, "rank": r, "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
                              "master": "%s:%s" % (os.environ.get("MASTER_ADDR"), os.environ.get("MASTER_PORT"))}))
        else:  # a failing rank 0 must not leave the others waiting forever (they wait here briefly)
            time.sleep(float(os.environ.get("USAC_BENCH_DRY_SLEEP", "0")))
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("USAC_BENCH_SAME_DEVICE"):  # rehearsal of the N > 1 path on a 1-GPU box
        local_rank = 0
    _DEV = local_rank
    # one hardware queue per in-flight batch (HIP's default is 4 per process: more contexts would share
    # queues and serialise behind each other's long kernels); set before the runtime initialises
    # (essential: a second, CU-masked stream per context for its root-order kernels)
    queues = args.pipeline * (2 if args.estimator == "essential" else 1)
    if queues > int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4):
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(queues, 32))
    import torch  # noqa: F401  (torch.distributed rendezvous; loads the process's HIP runtime first)
    import torch.distributed as dist

    import ransac_amd as usac
    from ransac_amd import synthetic

    if world > 1:
        dist.init_process_group("gloo")
    if args.cfg5:
        return cfg5_main(args, usac, synthetic, dist, torch, world, rank, local_rank)
    if args.sprt_exact:
        return cfg3_exact_main(args, usac, synthetic, dist, torch, world, rank, local_rank)
    fund = args.estimator == "fundamental"
    ess = args.estimator == "essential"
    napsac = args.sampler == "napsac"
    if fund or ess:
        pts, _, _ = synthetic.fundamental_points(n=args.points, inlier_ratio=0.3, seed=args.seed, normalized=ess)
    elif napsac:  # the cfg5 generator: inliers clustered (NAPSAC's premise), 20 %
        pts, _, _ = synthetic.homography_points(n=args.points, inlier_ratio=0.2, seed=args.seed,
                                                cluster=(500, 500, 150))
    else:
        pts, _, _ = synthetic.homography_points(n=args.points, inlier_ratio=0.3, seed=args.seed)
    dlt_mode = 0 if args.dlt == "thin" else 1
    est_id = usac.ESTIMATOR.Fundamental if fund else usac.ESTIMATOR.Essential if ess else usac.ESTIMATOR.Homography
    P = max(1, args.pipeline)
    # the N > 1 exchange keeps one ring slot per batch in flight
    assert world == 1 or P <= usac.Context.XRING, "at most %d batches in flight (exchange ring)" % usac.Context.XRING
    ctxs = [usac.Context(est_id, pts, device=local_rank) for _ in range(P)]
    for c in ctxs:
        c.set_dlt_mode(dlt_mode)
        c.set_score_chunks(args.chunks)
        if args.sampler == "prosac":  # points are quality-sorted (synthetic generator)
            c.set_device_sampler(usac.SAMPLER.Prosac)
        elif napsac:  # grid neighbours built on the device at context setup (not timed)
            c.set_device_sampler(usac.SAMPLER.Napsac)
    ctx = ctxs[0]
    for c in ctxs[1:]:  # in-pipeline timings from ctxs[0]'s batches (finish)
        c.set_timing(False)
    exchange = "none"
    if world > 1:  # the per-batch best-record exchange: RCCL all-gather on the context stream
        uid = [usac.Context.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        exchange = init_exchange(ctx, usac, dist, torch, world, rank, uid[0])
    rccl = rccl_report(ctx, exchange, dist, world, rank)

    def allgather(rec):
        if exchange == "rccl_allgather":
            return ctx.allgather_record(rec)
        buf = torch.frombuffer(bytearray(bytes(rec)), dtype=torch.uint8)
        out = [torch.zeros_like(buf) for _ in range(world)]
        dist.all_gather(out, buf)
        return [usac.Record.from_buffer_copy(bytes(o.numpy().tobytes())) for o in out]
    B = args.batch
    if args.sprt:
        for c in ctxs:
            c.set_sprt(True, seed=args.seed)
    models_per_hyp = 1.0
    timed_first = (args.warmup * world + rank) * B  # the first timed batch's first hypothesis
    if fund or ess:  # occupied model slots per sample of the first timed batch (the device stream)
        ctx.set_sprt(False)
        c0, _, _ = ctx.hypothesize_score(B=B, seed=args.seed, first_hyp=timed_first, thr=args.threshold)
        models_per_hyp = float((c0 >= 0).sum()) / B
        if args.sprt:
            ctx.set_sprt(True, seed=args.seed)

    def sync():
        for c in ctxs:
            c.sync()
        if torch.cuda.is_available():
            torch.cuda.synchronize(local_rank)

    def launch(i):
        first = (i * world + rank) * B
        ctxs[i % P].hypothesize_async(B, args.seed, first, args.threshold)
        if exchange == "rccl_allgather":
            # the batch best is all-gathered on ctx's exchange stream, ordered after this
            # batch's stream by an event: finish(i) then waits for batch i's exchange only
            ctx.exchange_best_async(ctxs[i % P], i % ctx.XRING)

    def finish(i):
        c = ctxs[i % P]
        if exchange == "rccl_allgather":
            best = usac.merge_records(ctx.exchange_best_wait(i % ctx.XRING))
        else:
            best = c.fetch_best()
            if world > 1:
                best = usac.merge_records(allgather(best))
        # the in-pipeline HIP-event times of the first context's batches only (the others record no
        # events: four event records, three elapsed-time queries and their Python wrapping per batch
        # are host time inside the loop, and the 0.11 ms cfg2 steps feel it)
        t = c.last_timings() if i % P == 0 else None
        return best, t

    def run(first_step, count, sink):
        # keep P batches in flight: batch i is launched before batch i - P + 1 is fetched
        for j in range(count):
            launch(first_step + j)
            if j >= P - 1:
                sink(*finish(first_step + j - P + 1))
        for j in range(max(0, count - P + 1), count):
            sink(*finish(first_step + j))

    # untimed device warm-up (clocks, caches, queues): batches of the same workload beyond every
    # timed index, until --prewarm-ms has passed; then the W warmup steps as before
    pre_batches = 0
    if args.prewarm_ms > 0 and torch.cuda.is_available():
        base = args.warmup + args.steps + 1000
        tw = time.perf_counter()
        while True:
            go = (time.perf_counter() - tw) * 1e3 < args.prewarm_ms
            if world > 1:  # every rank runs the same batches (each launch may be a collective)
                flag = torch.tensor([1 if go else 0], dtype=torch.int32)
                dist.all_reduce(flag, op=dist.ReduceOp.MIN)
                go = bool(flag.item())
            if not go:
                break
            run(base + pre_batches, 4 * P, lambda rec, t: None)
            pre_batches += 4 * P
    run(0, args.warmup, lambda rec, t: None)
    if world > 1:
        dist.barrier()
    sync()
    score_ms, solve_ms, batch_ms = [], [], []
    best_box = [None]
    first_box = []  # the first timed batch's merged record (checked against the oracle afterwards)

    def keep(rec, t):
        if t is not None:
            score_ms.append(t["score_ms"])
            solve_ms.append(t["solve_ms"])
            batch_ms.append(t["batch_ms"])
        if not first_box:
            first_box.append(rec)
        b = best_box[0]
        if b is None or not usac.record_better(b, rec):  # usac_merge_records([rec, b]) in Python
            best_box[0] = rec

    t0 = time.perf_counter()
    run(args.warmup, args.steps, keep)
    best = best_box[0]
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tested_per_batch = ctxs[(args.warmup + args.steps - 1) % P].sprt_tested() if args.sprt else None
    # roofline pass: the same batches one at a time (no overlap), so the per-kernel durations
    # are the kernels' own (what rocprofv3 reports for `bench.py --pipeline 1`)
    solo_score, solo_solve = [], []
    for i in range(max(5, min(args.steps, 20))):
        ctx.hypothesize_async(B, args.seed, ((args.warmup + args.steps + i) * world + rank) * B, args.threshold)
        ctx.fetch_best()
        t = ctx.last_timings()
        solo_score.append(t["score_ms"])
        solo_solve.append(t["solve_ms"])
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    # parity of the timed configuration on every rank (N > 1: each rank's own 256-sample slice, its
    # record also through the line's exchange), gathered to rank 0
    tk_all = None
    if world > 1:
        tk_first = rank * 256  # the stream's head, as at N = 1 (PROSAC's early subsets: SPRT accepts models there)
        own = timed_kernel_parity(usac, ctx, args.estimator, pts, args.threshold, dlt_mode, args.seed,
                                  bool(args.sprt), first_hyp=tk_first,
                                  xctx=ctx if exchange == "rccl_allgather" else None)
        tk_all = [None] * world
        dist.all_gather_object(tk_all, own)

    if rank == 0:
        total = world * args.steps * B
        value = total / elapsed
        n = args.points
        m = 7 if fund else 5 if ess else 4
        # N*S per scored model + m*4 + k*(36+8)
        if args.sprt:  # with SPRT, the bytes actually tested (16 B x tested points)
            bytes_per_hyp = 16.0 * tested_per_batch / B + m * 4 + models_per_hyp * (36 + 8)
        else:
            bytes_per_hyp = models_per_hyp * 16 * n + m * 4 + models_per_hyp * (36 + 8)
        avg_score_ms = float(np.mean(solo_score))
        avg_solve_ms = float(np.mean(solo_solve))
        achieved = bytes_per_hyp * B / (avg_score_ms * 1e-3) / 1e9
        # the dominant stage of a batch (solo HIP-event times): its kernels' VALU roofline
        stage = "solve" if avg_solve_ms > avg_score_ms else "score"
        other = "score" if stage == "solve" else "solve"
        stage_ms = {"score": avg_score_ms, "solve": avg_solve_ms}
        knames = {st: _stage_kernels(args.estimator, args.sprt, args.chunks, st) for st in ("score", "solve")}
        roof = None
        if not (fund or ess) and not args.sprt and stage == "score":  # cfg2: the score kernel alone (unchanged form)
            roof = valu_roofline(next(k for k in knames["score"] if "k_score" in k), n, B, avg_score_ms)
            if roof is not None:
                roof["stage"] = stage_roofline(knames["score"], n, B, avg_score_ms)
        if roof is None:
            roof = stage_roofline(knames[stage], n, B, stage_ms[stage])
        if roof is None:
            roof = {"bound": "valu", "achieved": None, "peak": SIMD_CYCLES_S, "unit": "SIMD-cycles/s", "frac": None,
                    "note": "no committed PMC summary (profiles/r*_summary.json) for these kernels and workload"}
        roof["other_stage"] = {"stage": other, "ms": stage_ms[other],
                               "roofline": stage_roofline(knames[other], n, B, stage_ms[other])}
        kshort = "+".join(k.replace("void ", "").replace("usac::", "").rstrip("(").replace(" ", "")
                          for k in knames[stage])
        roof.update({
            "traffic": roof.get("hbm", {}).get("traffic_bytes_per_launch"), "traffic_unit": "bytes/launch",
            "dominant_stage": stage,
            "kernel": kshort, "kernel_ms": stage_ms[stage], "hypotheses_per_launch": B, "sprt": bool(args.sprt),
            "sprt_points_tested_per_batch": tested_per_batch, "models_per_hypothesis": models_per_hyp,
            "algorithmic_bytes_per_hypothesis": bytes_per_hyp,
            "algorithmic_equiv_gbs": achieved,
            "note": "frac = VALU-busy SIMD-cycles per launch / the dominant stage's HIP-event time / (1024 SIMDs x "
                    "2.4 GHz): for the cfg2 score kernel SQ_INSTS_VALU x the ISA hot loop's mean issue cost per "
                    "opcode as measured on an MI355X (issue_model; frac_guide = the guide's plain 2 / packed 4 "
                    "cycles; frac_x4 = the SQ_ACTIVE_INST_VALU x 4 form), for the other stages SQ_ACTIVE_INST_VALU x 4 summed over the "
                    "stage's kernels; other_stage: the same for the other stage of the batch.  The score kernel is "
                    "fp32-VALU-issue bound with its point records L2/scalar-cache resident, so `hbm` (counter-"
                    "measured bytes) is a small fraction of HBM peak; algorithmic_equiv_gbs = SURVEY §8(d) bytes "
                    "(16 B x N per hypothesis) / kernel time, a re-read-equivalent rate, not a roofline fraction",
            "score_kernel_ms": avg_score_ms,
            # (the first context's timed batches; None when none of them fell in the timed steps)
            "solve_kernel_ms": avg_solve_ms, "kernel_ms_in_pipeline": float(np.mean(score_ms)) if score_ms else None,
            "solve_kernel_ms_in_pipeline": float(np.mean(solve_ms)) if solve_ms else None,
            "batch_device_ms_in_pipeline": float(np.mean(batch_ms)) if batch_ms else None})
        smp_name = {"prosac": "Prosac (reference subset schedule, T_N = 200000)",
                    "napsac": "Napsac (grid neighbours, cell 50, built on the device)"}.get(args.sampler, "Uniform")
        out = {
            "metric": "model hypotheses/sec (sample+solve+score) and inlier-count match vs ref",
            "value": value,
            "unit": "hypotheses/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup, "prewarm": {"ms": args.prewarm_ms, "batches": pre_batches},
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("synthetic (SURVEY §8(d) cfg3 generator: two views, 30% inliers, 0.5 px noise)" if fund else
                     "synthetic (SURVEY §8(d) cfg4 generator: cfg3 geometry in K^-1-normalised coordinates)" if ess
                     else "synthetic (cfg5 generator: 20% inliers clustered around (500, 500), r = 150 px, uniform "
                          "outliers)" if napsac
                     else "synthetic (SURVEY §8(d) cfg2 generator: 30% inliers, 1 px noise, 70% uniform outliers)"),
            "config": {"workload": ("cfg3%s: Fundamental_estimator (7-pt, oriented filter, Sampson) + "
                                    "%s sampler (device stream), %d correspondences, %d-hypothesis batch per "
                                    "GPU, %.3f models/sample" % (" + batch SPRT" if args.sprt else " without SPRT",
                                                                 smp_name, n, B, models_per_hyp)) if fund else
                                   ("cfg4%s: Essential_estimator (5-pt, cheirality, epipolar distance) + %s "
                                    "sampler (device stream), %d correspondences, %d-hypothesis batch per GPU, "
                                    "%.3f models/sample" % (" + batch SPRT" if args.sprt else "", smp_name, n, B,
                                                            models_per_hyp)) if ess else
                                   ("%s%s: Homography_estimator (4-pt DLT, %s) + %s sampler (device "
                                    "stream), %d correspondences, %d-hypothesis batch per GPU" %
                                    ("cfg5 batches (throughput, no LO)" if napsac else "cfg2",
                                     " + batch SPRT" if args.sprt else "", args.dlt, smp_name, n, B)),
                       "sampler": args.sampler,
                       "n_points": n, "batch_per_gpu": B, "threshold": args.threshold,
                       "score_chunks": args.chunks, "batches_in_flight": P,
                       "parallelism": "hypothesis-sharded x%d" % world, "exchange": exchange},
            "roofline": roof,
            "best": {"inliers": int(best.inliers), "hyp_index": int(best.hyp_index)},
        }
        out["config"]["rccl"] = rccl
        par = parity_check(usac, args.estimator, pts, args.threshold, dlt_mode,
                           samples=ctx.draw_samples(256, args.seed) if napsac else None)
        if world == 1:
            par["timed_kernel"] = timed_kernel_parity(usac, ctx, args.estimator, pts, args.threshold, dlt_mode,
                                                      args.seed, bool(args.sprt))
        else:
            par["timed_kernel"] = tk_all[0]
            par["ranks"] = ranks_parity(usac, tk_all, exchange)
        if not args.sprt:  # batch SPRT decisions depend on each rank's batch state: ranks_parity covers them
            par["first_timed_batch"] = first_batch_parity(usac, ctx, args.estimator, pts, args.threshold, dlt_mode,
                                                          args.seed, B, args.warmup, world, first_box[0],
                                                          cpu_info()[2])
        par["ok"] = bool(par["inlier_counts_equal"] and par["scores_bit_equal"] and par["timed_kernel"]["ok"] and
                         par.get("ranks", {}).get("ok", True) and par.get("first_timed_batch", {}).get("ok", True))
        out["parity"] = par
        if fund or ess:  # occupied model slots per sample of the first timed batch (beside the value)
            out["models_per_hypothesis"] = models_per_hyp
        if args.cpu_seconds > 0:
            if args.sprt:  # the same hypotheses through the oracle (same samples, models, SPRT decisions)
                out["cpu_baseline"] = cpu_baseline_batch_sprt(usac, ctx, args.estimator, pts, args.threshold, dlt_mode,
                                                              args.seed, timed_first, args.cpu_seconds)
            else:
                out["cpu_baseline"] = cpu_baseline(args.estimator, pts, args.threshold, dlt_mode, args.cpu_seconds)
            out["gpu_over_cpu"] = value / out["cpu_baseline"]["value"]
        print(json.dumps(out), flush=True)
    if world > 1:  # the other ranks wait for rank 0's checks and CPU baseline before tearing down
        dist.barrier()
    for c in ctxs:
        c.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
