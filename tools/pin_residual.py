"""explain the notebook-pin A residual (CPU only; test infrastructure).

For every (cell, rounds) point of the pin (Threshold-checkpoint.ipynb cells 16 / 20 / 25, printed
fits at notebook lines 577-587, 781-785, 876-900) and in particular the three held-out A outliers
(cell 16 R15, cell 20 R30, cell 25 R25), from the engine's held-out 25x counts
(profiles/r05/pin/heldout_counts.json, seed 0x55EED, ADOPTED hypotheses):

(a) the parametric bootstrap of the notebook's experiment (binomial counts at the notebook's sample
    sizes, refit with the notebook's ThresholdEst, lines 71-120): how often the refit is degenerate
    (p_c outside [p_min / 2, 2 p_max], a distance fit d <= 0, d not increasing with code size) and
    how sensitive it is to curve_fit's initial guess (the same replica refit from 4 other p0);
    the (ln A, ln p_c) ridge of the replicas and where the printed pair sits across it;
(b) the per-(code, p) logical error rate the printed (A, p_c) implies (WER = A (p / p_c)^(d / 2)
    with the engine fit's distances d, inverted through the WER transform), against the engine's
    measured rate and its 95 % Wilson interval;
(c) a verdict per point: "fit artefact" when the printed pair is on the replicas' ridge (its
    across-ridge residual inside the central 95 %) and the implied rates are within 3 sigma of the
    engine's, "decoder statistics" otherwise.

    python tools/pin_residual.py [out.json]
"""
import json
import math
import os
import sys
import warnings

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import notebook_pin as nbp  # noqa: E402

from scipy.optimize import curve_fit  # noqa: E402

OUTLIERS = [(16, 15), (20, 30), (25, 25)]
P0_ALT = [(0.02, 0.01), (0.08, 1.0), (0.03, 0.003), (0.06, 0.03)]
DRAWS = 400


def fit_full(P, WER, p0=(0.04, 0.1)):
    """ThresholdEst (notebook lines 71-120) returning (A, p_c, ds); p0 of the empirical fit."""
    ds = []
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for row in WER:
            popt, _ = curve_fit(nbp._fit_distance, np.log10(P), np.log10(row + 1e-6), p0=(0.08, 3))
            ds.append(popt[1])
        X = np.vstack([np.tile(P, len(WER)), np.repeat(np.asarray(ds), len(P))])
        popt, _ = curve_fit(nbp._emperical_fit, X, WER.reshape(-1), p0=p0, maxfev=20000)
    return float(popt[1]), float(popt[0]), [float(d) for d in ds]


def ler_from_wer(w, K, R):
    """Inverse of notebook_pin.wer_current (q <= 1/2 branch): WER -> per-sample logical failure rate."""
    lo = np.clip(np.asarray(w, dtype=np.float64), 0.0, 0.5)
    q = (1.0 - (1.0 - 2.0 * lo) ** R) / 2.0
    return 1.0 - (1.0 - q) ** K


def wilson(k, n, z=1.96):
    ph = k / n
    den = 1 + z * z / n
    c = (ph + z * z / (2 * n)) / den
    h = z * math.sqrt(ph * (1 - ph) / n + z * z / (4 * n * n)) / den
    return c - h, c + h


def point(cell, R, c, rng_seed):
    P = nbp.cell_p_list(cell)
    K = c["K"]
    S = c["samples"]
    fail = np.asarray(c["fail"], dtype=np.float64)
    fp = fail / S
    wer = np.vstack([nbp.wer_current(fail[i], S, K[i], R) for i in range(3)])
    A_e, pc_e, d_e = fit_full(P, wer)
    A0, pc0, line = nbp.PRINTED[cell][R]
    ns = nbp.cell_samples(cell, R)
    rng = np.random.default_rng(rng_seed)
    fits, degen, sens, failed = [], 0, 0, 0
    for _ in range(DRAWS):
        cnt = rng.binomial(ns, np.clip(fp, 0, 1))
        w = np.vstack([nbp.wer_current(cnt[i], ns, K[i], R) for i in range(3)])
        if not np.all(np.isfinite(w)):
            failed += 1
            continue
        try:
            A, pc, ds = fit_full(P, w)
        except (RuntimeError, ValueError, TypeError):
            failed += 1
            continue
        fits.append((A, pc))
        bad = not (P[0] / 2 <= pc <= 2 * P[-1]) or min(ds) <= 0 or not (ds[0] < ds[1] < ds[2])
        degen += bad
        moved = False
        for p0 in P0_ALT:
            try:
                A2, pc2, _ = fit_full(P, w, p0)
                moved |= abs(A2 - A) > 0.01 * abs(A) or abs(pc2 - pc) > 0.01 * abs(pc)
            except (RuntimeError, ValueError, TypeError):
                moved = True
        sens += moved
    F = np.asarray(fits)
    lnA, lnpc = np.log(F[:, 0]), np.log(F[:, 1])
    b, a = np.polyfit(lnpc, lnA, 1)  # the replicas' ridge: ln A = a + b ln p_c
    res = lnA - (a + b * lnpc)
    r0 = math.log(A0) - (a + b * math.log(pc0))
    res_pct = nbp.mid_percentile(r0, res)
    # (b) the rates the printed pair implies, with the engine fit's distances
    imp, rows = [], []
    worst = 0.0
    for i in range(3):
        w_imp = A0 * (P / pc0) ** (np.asarray(d_e[i]) / 2)
        l_imp = ler_from_wer(w_imp, K[i], R)
        for j, p in enumerate(P):
            k = int(fail[i, j])
            lo, hi = wilson(k, S)
            sd = math.sqrt(max(fp[i, j] * (1 - fp[i, j]), 1e-12) / S)
            z = (float(l_imp[j]) - fp[i, j]) / sd
            worst = max(worst, abs(z))
            rows.append({"code": i, "p": float(p), "engine_ler": fp[i, j], "engine_ci95": [lo, hi],
                         "implied_ler": float(l_imp[j]), "z": z})
    # the same with each code's slope d_c chosen to fit the engine's rates best (log least squares):
    # can ANY distances make the printed (A, p_c) reproduce the engine's per-code rates?
    best = []
    for i in range(3):
        y = np.log(np.clip(wer[i], 1e-12, None)) - math.log(A0)
        x = np.log(P / pc0) / 2
        d_fit = float(np.sum(x * y) / np.sum(x * x))
        w_imp = A0 * (P / pc0) ** (d_fit / 2)
        best.append({"code": i, "d_best": d_fit, "d_engine": d_e[i],
                     "implied_over_engine": [float(a / b) for a, b in zip(ler_from_wer(w_imp, K[i], R), fp[i])]})
    frac_in = float(np.mean([lo <= r["implied_ler"] <= hi for r in rows for lo, hi in [r["engine_ci95"]]]))
    mean_ratio = float(np.mean([r["implied_ler"] / max(r["engine_ler"], 1e-12) for r in rows]))
    on_ridge = 0.025 <= res_pct <= 0.975
    verdict = "fit artefact" if (on_ridge and worst <= 3.0) else ("fit artefact (ridge)" if on_ridge else "decoder statistics")
    return {
        "cell": cell, "rounds": R, "printed": {"A": A0, "p_c": pc0, "notebook_line": line},
        "engine_fit": {"A": A_e, "p_c": pc_e, "d": d_e},
        "bootstrap": {"draws": DRAWS, "failed": failed, "ok": len(F),
                      "A_pct": nbp.mid_percentile(A0, F[:, 0]), "p_c_pct": nbp.mid_percentile(pc0, F[:, 1]),
                      "degenerate_frac": degen / max(len(F), 1),
                      "p0_sensitive_frac": sens / max(len(F), 1),
                      "ridge": {"slope_dlnA_dlnpc": float(b), "intercept": float(a),
                                "corr": float(np.corrcoef(lnpc, lnA)[0, 1]),
                                "printed_residual": r0, "printed_residual_pct": res_pct,
                                "residual_sd": float(np.std(res))}},
        "implied_best_slopes": best,
        "implied_vs_engine": {"max_abs_z": worst, "frac_inside_engine_ci95": frac_in,
                              "mean_implied_over_engine": mean_ratio, "points": rows},
        "verdict": verdict,
    }


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r06", "pin", "A_residual.json")
    src = json.load(open(os.path.join(ROOT, "profiles", "r05", "pin", "heldout_counts.json")))
    cells = src["hypotheses"]["adopted"]["cells"]
    res = []
    for cell in (16, 20, 25):
        for R in nbp.CELLS[cell]["rounds"]:
            c = cells[str(cell)]["counts"][str(R)]
            r = point(cell, R, c, 17 + R + cell)
            res.append(r)
            b = r["bootstrap"]
            print(f"cell {cell} R{R:2d}: A pct {b['A_pct']:.3f} p_c pct {b['p_c_pct']:.3f} degen {b['degenerate_frac']:.2f} "
                  f"p0-sens {b['p0_sensitive_frac']:.2f} ridge corr {b['ridge']['corr']:.3f} resid pct "
                  f"{b['ridge']['printed_residual_pct']:.3f} | implied/engine {r['implied_vs_engine']['mean_implied_over_engine']:.2f}"
                  f" max|z| {r['implied_vs_engine']['max_abs_z']:.1f} -> {r['verdict']}", flush=True)
            for bb in r["implied_best_slopes"]:
                print(f"      code {bb['code']}: d_engine {bb['d_engine']:.2f} d_best {bb['d_best']:.2f} implied/engine "
                      + " ".join(f"{v:.2f}" for v in bb["implied_over_engine"]))
    resid = [r["bootstrap"]["ridge"]["printed_residual_pct"] for r in res]
    summary = {"what": __doc__.strip().splitlines()[0], "source": "profiles/r05/pin/heldout_counts.json (seed 0x55eed)",
               "outliers": [f"cell {c} R{R}" for c, R in OUTLIERS],
               "A_uniformity": nbp.uniformity([r["bootstrap"]["A_pct"] for r in res]),
               "p_c_uniformity": nbp.uniformity([r["bootstrap"]["p_c_pct"] for r in res]),
               "ridge_residual_uniformity": nbp.uniformity(resid),
               "points": res}
    os.makedirs(os.path.dirname(out_path), exist_ok=True)
    with open(out_path, "w") as f:
        json.dump(summary, f, indent=1, default=float)
    print("A:", summary["A_uniformity"])
    print("p_c:", summary["p_c_uniformity"])
    print("ridge residual:", summary["ridge_residual_uniformity"])


if __name__ == "__main__":
    main()
