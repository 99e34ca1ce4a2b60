"""The batch SPRT's decisions against the oracle (kernels_sprt.hip): every occupied model slot of
the last batch, walked by the oracle with the reference's fp64 lambda product (sprt.hpp:209-234)
from the pool position the device started that model at, with the batch's (epsilon, delta, A)."""
import numpy as np


def batch_sprt_vs_oracle(oracle, ctx, okind, pts, thr, samples, counts, pool_seed, m):
    S = ctx.spk
    B = len(samples)
    (eps, delta, A), starts = ctx.batch_sprt_info(B * S)
    est = oracle.Estimator(okind, pts)
    om, onm = est.estimate_batch(samples)
    om = np.asarray(om, np.float32).reshape(B, -1, 9)
    if S == 3:
        occ = (np.arange(3)[None, :] < onm[:, None]).reshape(-1)
    else:
        occ = (onm == 1) if okind == oracle.ESSENTIAL else np.ones(B, bool)
    models = om.reshape(-1, 9)[: B * S][occ] if S == 3 else om[:, 0][occ]
    pool, _ = oracle.sprt_pool(pool_seed, okind, len(pts), m)
    good, cnt, tested = oracle.sprt_fixed_batch(est, pool, thr, models, starts[occ], eps, delta, A)
    return {"device": np.asarray(counts)[occ], "oracle": cnt, "accepted": int(good.sum()), "models": int(occ.sum()),
            "oracle_tested": int(tested.sum()), "empty_slots_ok": bool((np.asarray(counts)[~occ] < 0).all()) and
            bool((starts[~occ] == 0xFFFFFFFF).all())}  # usac_batch_sprt_info: an empty slot has no start
