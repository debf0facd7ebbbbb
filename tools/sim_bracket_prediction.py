"""CPU simulation (numpy): could the top-k step skip its sampled bracket by predicting the k-th |t|
from the previous steps of the same name?  Top-k 1 % + residual error feedback on n = 2^20,
several gradient streams; the predictor extrapolates log T linearly from the last two exact k-th
keys, the band half-width is h = max(h_min, c * recent prediction error + pad), and a step is
predicted only when h <= h_max and the band's expected candidate count (the density of |t| around
T, measured on the previous step) stays under 0.6 k -- the sampled bracket's band holds about
0.45 k.  A miss (the k-th key outside the band, or more candidates than the list holds) is what
the engine would pay for with its exact fallback.  Results are recorded in DESIGN.md §4.
usage: python tools/sim_bracket_prediction.py
"""
import math

import numpy as np


def run(scen, rng, n=1 << 20, ratio=0.01, steps=120, hmin=0.004, c=4.0, pad=0.002, hmax=0.05):
    k = int(n * ratio)
    g0 = rng.standard_normal(n).astype(np.float32)
    scales = np.exp(rng.standard_normal(n // 4096)).repeat(4096).astype(np.float32)
    pool = [rng.standard_normal(n).astype(np.float32) for _ in range(16)] if scen.startswith("rot") else None
    r = np.zeros(n, np.float32)
    t1 = t2 = 0.0
    e_prev = 1.0
    use, lo, hi = False, 0.0, 0.0
    st = {"predicted": 0, "misses": 0, "mean_cand_over_k": 0.0}
    for s in range(steps):
        if scen == "fixed_g":                    # the same gradient every step
            g = g0
        elif scen == "fresh_g":                  # a new gradient every step
            g = rng.standard_normal(n).astype(np.float32)
        elif scen == "scale_jump":               # gradients 3x larger from step 60 on
            g = rng.standard_normal(n).astype(np.float32) * (3.0 if s >= 60 else 1.0)
        elif scen == "layers":                   # per-4096-element scales (a bucket of tensors)
            g = rng.standard_normal(n).astype(np.float32) * scales
        elif scen == "decay":                    # shrinking gradients
            g = rng.standard_normal(n).astype(np.float32) * (0.97 ** s)
        else:                                    # rotN: N fixed gradients in turn
            g = pool[s % int(scen[3:])]
        t = r + g
        a = np.abs(t)
        T = float(np.partition(a, n - k)[n - k])
        ok = True
        if use:
            st["predicted"] += 1
            ncand = int(((a >= lo) & (a <= hi)).sum())
            nsure = int((a > hi).sum())
            ok = nsure <= k and nsure + ncand >= k and ncand <= 2 * k + 65536 * k // 671088
            st["misses"] += not ok
            st["mean_cand_over_k"] += ncand / k
        idx = np.argpartition(-a, k)[:k]
        r = t.copy()
        r[idx] = 0
        e = abs(math.log(T) - math.log(t1 * t1 / t2)) if t1 > 0 and t2 > 0 else 1.0
        emax = max(e, e_prev)
        e_prev = e
        if use and not ok:
            t1 = t2 = 0.0
            e_prev = emax = 1.0
        t2, t1 = t1, T
        use = False
        if t1 > 0 and t2 > 0:
            p = t1 * t1 / t2
            h = max(hmin, c * emax + pad)
            rho = ((a >= T * math.exp(-0.03)) & (a <= T * math.exp(0.03))).sum() / 0.06
            use = h <= hmax and rho * 2 * h <= 0.6 * k
            lo, hi = p * math.exp(-h), p * math.exp(h)
    if st["predicted"]:
        st["mean_cand_over_k"] = round(st["mean_cand_over_k"] / st["predicted"], 3)
    return st


if __name__ == "__main__":
    rng = np.random.default_rng(1)
    for scen in ("fixed_g", "rot3", "rot8", "rot16", "fresh_g", "scale_jump", "layers", "decay"):
        print(scen, run(scen, rng), flush=True)
