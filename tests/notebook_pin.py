"""Pin of the BP / BP+OSD arithmetic against outputs the reference itself printed.

Test infrastructure (not product code).  The reference's BP and OSD live in the
absent third-party ``ldpc`` / ``bposd`` packages; the only outputs the reference
holds that those packages produced are the threshold fits printed by
``.ipynb_checkpoints/Threshold-checkpoint.ipynb`` (phenomenological noise, real
``ldpc.bp_decoder`` + ``bposd.bposd_decoder``).  Three of its cells run on codes
this repository holds exactly:

* cell 16 — LP ``[[544,80]] [[714,100]] [[1020,136]]`` (``codes_lib/LP_Matg8_L{16,21,30}``),
  ``eval_p = linspace(0.02, 0.035, 6)``, rounds {6,10,15,20,25,30},
  ``int(4000*3/R)`` samples (notebook lines 665-671, printed fits 577-587);
* cell 20 — the same codes, ``linspace(0.015, 0.03, 6)``, rounds {20,25,30},
  ``int(12000*3/R)`` samples (lines 827-834, printed 781-785);
* cell 25 — toric d5/d9/d13 = ``hgp(ring_code(d), ring_code(d))`` (cell 9, line 329),
  ``linspace(0.008, 0.02, 6)``, rounds {6,...,30}, ``int(10000*3/R)`` samples
  (lines 978-985, printed 876-900).

Every point is ``CodeFamilyPhenlThreshold`` (notebook lines 127-170):
``CodeSimulator_Phenon`` with ``q`` left at 0 (``src/Simulators.py:195``),
decoder1 = ``BPDecoder`` on ``[h | I]``, priors ``2p/3`` on every column,
``max_iter = int(N/30)``, min-sum α 0.625; decoder2 = ``BPOSD_Decoder``
OSD-E(10), ``max_iter = int(N/10)``; then the notebook's own ``ThresholdEst``
(lines 71-120) fits ``(A, p_c)``.

The printed fits are one draw from the reference's sampling distribution.  The
engine's failure probabilities, estimated at many times the notebook's sample
counts, define that distribution under the hypothesis "same decoder
statistics"; a parametric bootstrap (binomial counts at the notebook's sample
sizes, refit with the notebook's fit) gives the 95 % band each printed value
must fall in.

The WER transform: the notebook ran even round counts, which the current
``CodeSimulator_Phenon.WordErrorRate`` rejects (``assert int(num_rounds)%2 == 1``,
``src/Simulators.py:353``), so the printed fits were made with the version kept
as a comment at ``src/Simulators.py:341-351``: per-cycle logical rate
``(1-(1-2·LER)^(1/R))/2``, then ``WER = 1-(1-per_cycle)^(1/K)``.  Both are
restated (``wer_commented`` and ``wer_current``) so the test can report which
one the printed values are consistent with.
"""
from __future__ import annotations

import math
import warnings

import numpy as np

# ----------------------------------------------------------------- printed fits
# (cell, rounds) -> (A, p_c, notebook line of the printed "A: ... p_c: ..." text)
PRINTED = {
    16: {6: (0.017049050841283525, 0.06337604972427469, 577),
         10: (0.006395614537064315, 0.05011620442766196, 579),
         15: (0.0029650182854605435, 0.042952768244995554, 581),
         20: (0.003488304092697116, 0.04391058695786237, 583),
         25: (0.00035028650686427337, 0.028826365997509887, 585),
         30: (0.26663113712874625, 0.09591491905342583, 587)},
    20: {20: (0.003031945260488044, 0.04334163091869549, 781),
         25: (0.011283027790160122, 0.055145595306794075, 783),
         30: (0.0014778297920826672, 0.037340038191445275, 785)},
    25: {6: (0.10811638601355365, 0.04966058344937042, 876),
         10: (0.03261492761610603, 0.030333299465439507, 878),
         15: (0.02439441279823083, 0.02538680708170507, 880),
         20: (0.013969992505888488, 0.020702275280256255, 882),
         25: (0.00822491914697463, 0.016883796009653614, 884),
         30: (0.007204022239674292, 0.015562687486884634, 900)},
}

CELLS = {
    16: {"codes": ["LP_Matg8_L16_Dmin12", "LP_Matg8_L21_Dmin16", "LP_Matg8_L30_Dmin20"],
         "p": (0.02, 0.035, 6), "num_samples": 4000, "rounds": [6, 10, 15, 20, 25, 30]},
    20: {"codes": ["LP_Matg8_L16_Dmin12", "LP_Matg8_L21_Dmin16", "LP_Matg8_L30_Dmin20"],
         "p": (0.015, 0.03, 6), "num_samples": 12000, "rounds": [20, 25, 30]},
    25: {"codes": ["toric_d5", "toric_d9", "toric_d13"],
         "p": (0.008, 0.02, 6), "num_samples": 10000, "rounds": [6, 10, 15, 20, 25, 30]},
}


def cell_p_list(cell: int) -> np.ndarray:
    a, b, k = CELLS[cell]["p"]
    return np.linspace(a, b, k)


def cell_samples(cell: int, rounds: int) -> int:
    """``int(num_samples*3/sweep_num_round)`` (notebook lines 671, 833, 984)."""
    return int(CELLS[cell]["num_samples"] * 3 / rounds)


def ring_code(d: int) -> np.ndarray:
    """``ldpc.codes.ring_code(d)``: the d×d cyclic repetition-code check matrix."""
    h = np.zeros((d, d), dtype=np.uint8)
    for i in range(d):
        h[i, i] = 1
        h[i, (i + 1) % d] = 1
    return h


def cell_code(name: str):
    """The code objects of the notebook's cells 7 (LP) and 9 (toric)."""
    from qldpc_fault_tolerance_amd import codes

    if name.startswith("toric_d"):
        d = int(name[len("toric_d"):])
        return codes.hgp(ring_code(d), ring_code(d), name=name)
    return codes.get_code(name)


def decoder_params(N: int) -> dict:
    """``CodeFamilyPhenlThreshold`` decoder settings (notebook lines 137-158)."""
    return {"max_iter1": int(N / 30), "max_iter2": int(N / 10), "alpha": 0.625, "osd_order": 10}


# Hypotheses about what the notebook-era run did differently from the drop-in defaults
# (VERDICT r03 item 1).  q_frac: syndrome-flip probability q = q_frac·p in
# CodeSimulator_Phenon (src/Simulators.py:192 defaults q = 0; :203 says "The syndrom error prob
# equals 2/3 p for depolarizing noise", and decoder1's priors are 2p/3 on the syndrome columns,
# notebook lines 137-145).  round_shift: noisy rounds run = R - 1 + round_shift (an older
# _single_run that looped num_rounds times).  osd: the final-round OSD method / order.
HYPOTHESES = {
    "H0_q0": {"q_frac": 0.0, "round_shift": 0, "osd": ("osd_e", 10)},
    "Hq_2p3": {"q_frac": 2.0 / 3.0, "round_shift": 0, "osd": ("osd_e", 10)},
    "Hq_p": {"q_frac": 1.0, "round_shift": 0, "osd": ("osd_e", 10)},
    "Hrounds_plus1": {"q_frac": 0.0, "round_shift": 1, "osd": ("osd_e", 10)},
    "Hosd_cs10": {"q_frac": 0.0, "round_shift": 0, "osd": ("osd_cs", 10)},
    "Hosd0": {"q_frac": 0.0, "round_shift": 0, "osd": ("osd0", 0)},
}

# Adopted (profiles/r04/pin/hypotheses.json): the notebook's execution counts put the toric cell 25
# (In [30]) BEFORE the definition of CodeFamilyPhenlThreshold it calls (cell 3, In [50]) and the LP
# cells 16 / 20 (In [56], In [62]) after it, so the two groups ran different simulator states.  The
# LP cells match syndrome flips at q = 2p/3 (the rate src/Simulators.py:203 names, and decoder1's
# prior on the syndrome columns): the notebook's fit at the engine's rates gives p_c 0.0617 / 0.0500 /
# 0.0461 / 0.0440 against the printed 0.0634 / 0.0501 / 0.0430 / 0.0439 (R = 6-20), where q = 0 gives
# 0.110 / 0.069 / 0.058 / 0.056.  The toric cell matches q = 0 (0.0477 / 0.0344 / 0.0254 / 0.0214 vs
# 0.0497 / 0.0303 / 0.0254 / 0.0207); q = 2p/3 puts 4 of its 6 printed p_c above the 93rd percentile.
ADOPTED = {16: "Hq_2p3", 20: "Hq_2p3", 25: "H0_q0"}

# Post-hoc selection.  ADOPTED was picked per cell group (LP cells 16 / 20 share
# one hypothesis, the toric cell 25 another) from the 6 HYPOTHESES after seeing the seed-0x5EED
# counts: 6 x 6 = 36 combinations, the Bonferroni factor of every p-value of that selection run.
# HELDOUT_SEED draws a fresh 25x sample under ADOPTED, fixed before those counts existed (round 5);
# its p-values are pre-registered and need no correction.
SELECTION_SEED = 0x5EED
HYPOTHESIS_COMBINATIONS = len(HYPOTHESES) ** 2
HELDOUT_SEED = 0x5EED + 0x50000


def bonferroni(p: float, m: int = HYPOTHESIS_COMBINATIONS) -> float:
    """Bonferroni-corrected p-value over ``m`` hypothesis combinations."""
    return float(min(1.0, m * p)) if p == p else p


# ------------------------------------------------------------- WER transforms
def wer_commented(error_count, num_samples, K, num_rounds):
    """``src/Simulators.py:341-351`` (commented out today; the version the notebook's even R ran)."""
    ler = np.asarray(error_count, dtype=np.float64) / num_samples
    with np.errstate(invalid="ignore"):
        per_cycle = (1.0 - (1 - 2 * ler) ** (1 / num_rounds)) / 2
        return 1.0 - (1 - per_cycle) ** (1 / K)


def wer_current(error_count, num_samples, K, num_rounds):
    """``src/Simulators.py:353-360`` without its odd-R assert."""
    ler = np.asarray(error_count, dtype=np.float64) / num_samples
    q = 1.0 - (1 - ler) ** (1 / K)
    with np.errstate(invalid="ignore"):
        lo = (1.0 - (1 - 2 * q) ** (1 / num_rounds)) / 2
        hi = (1.0 + (-1 + 2 * np.abs(q)) ** (1 / num_rounds)) / 2
    return np.where(q <= 0.5, lo, hi)


WER_FORMULAS = {"commented": wer_commented, "current": wer_current}


# --------------------------------------------------------- the notebook's fit
def _fit_distance(logp, A, d):
    """Notebook cell 1 ``FitDistance`` (line 60-62): log-space, unlike ``src/Simulators.py:701``."""
    return A + (d / 2) * logp


def _emperical_fit(xdata_tuple, pc, A):
    """Notebook cell 1 ``EmpericalFit`` (lines 55-58)."""
    p, d = xdata_tuple
    return A * (p / pc) ** (d / 2)


def threshold_est(sweep_p_list, sweep_pl_total_list):
    """The notebook's ``ThresholdEst`` (lines 71-120) without the plot: returns ``(A, p_c)``.

    Per code a log-space distance fit (p0 (0.08, 3), +1e-6 offset), then the
    empirical ``A (p/p_c)^(d/2)`` fit over all points (p0 (0.04, 0.1)) on the
    raw rates.  Raises on a failed fit, as ``curve_fit`` does.
    """
    from scipy.optimize import curve_fit

    P = np.asarray(sweep_p_list, dtype=np.float64)
    PL = np.asarray(sweep_pl_total_list, dtype=np.float64)
    num_p, num_code = len(P), len(PL)
    ds = []
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for row in PL:
            popt, _ = curve_fit(_fit_distance, np.log10(P), np.log10(row + 1e-6), p0=(0.08, 3))
            ds.append(popt[1])
        X = np.vstack([np.tile(P, num_code), np.repeat(np.asarray(ds), num_p)])
        popt, _ = curve_fit(_emperical_fit, X, PL.reshape(num_p * num_code), p0=(0.04, 0.1))
    return float(popt[1]), float(popt[0])


# ------------------------------------------------------------------- bootstrap
def bootstrap_band(fail_prob, K_list, p_list, samples: int, rounds: int, formula="commented", draws=400,
                   seed=0, level=0.95):
    """Parametric bootstrap of the notebook's experiment at one round count.

    ``fail_prob[c][i]``: the engine's failure probability of code c at p_i.
    Draws binomial counts at the notebook's ``samples``, maps them through the
    WER transform and the notebook's fit.  Returns a dict with the band of A and
    of p_c (central ``level``), every successful fit, and the failed-fit count.
    """
    rng = np.random.default_rng(seed)
    f = WER_FORMULAS[formula]
    fits, failed = [], 0
    fp = np.clip(np.asarray(fail_prob, dtype=np.float64), 0.0, 1.0)
    for _ in range(int(draws)):
        cnt = rng.binomial(samples, fp)
        wer = np.vstack([f(cnt[c], samples, K_list[c], rounds) for c in range(len(K_list))])
        if not np.all(np.isfinite(wer)):
            failed += 1
            continue
        try:
            fits.append(threshold_est(p_list, wer))
        except (RuntimeError, ValueError, TypeError):
            failed += 1
    fits = np.asarray(fits, dtype=np.float64).reshape(-1, 2)
    lo_q, hi_q = (1 - level) / 2, 1 - (1 - level) / 2
    out = {"fits": fits, "failed": failed, "draws": int(draws)}
    if len(fits):
        out["A"] = (float(np.quantile(fits[:, 0], lo_q)), float(np.quantile(fits[:, 0], hi_q)))
        out["p_c"] = (float(np.quantile(fits[:, 1], lo_q)), float(np.quantile(fits[:, 1], hi_q)))
    return out


def inside(value: float, band) -> bool:
    return band is not None and band[0] <= value <= band[1]


def percentile_of(value: float, samples) -> float:
    s = np.sort(np.asarray(samples, dtype=np.float64))
    if len(s) == 0:
        return math.nan
    return float(np.searchsorted(s, value, side="right") / len(s))


def mid_percentile(value: float, samples) -> float:
    """Mid-rank percentile ``(#below + #equal/2 + 1/2) / (n + 1)``: never 0 or 1, so a
    printed value beyond every bootstrap replica still has a finite two-sided p."""
    s = np.asarray(samples, dtype=np.float64)
    if len(s) == 0:
        return math.nan
    below = float(np.sum(s < value))
    eq = float(np.sum(s == value))
    return (below + eq / 2 + 0.5) / (len(s) + 1)


def uniformity(pcts) -> dict:
    """Combined test that percentiles are U(0,1) (the printed values drawn from the engine's
    sampling distribution).  KS against the uniform CDF, and Fisher's method on the two-sided
    per-point p-values ``2 min(u, 1-u)``."""
    from scipy import stats

    u = np.asarray([x for x in pcts if np.isfinite(x)], dtype=np.float64)
    if len(u) == 0:
        return {"n": 0, "ks_p": math.nan, "fisher_p": math.nan}
    ks = stats.kstest(u, "uniform")
    two = np.clip(2 * np.minimum(u, 1 - u), 1e-12, 1.0)
    chi = float(-2 * np.sum(np.log(two)))
    return {"n": int(len(u)), "ks_stat": float(ks.statistic), "ks_p": float(ks.pvalue),
            "fisher_chi2": chi, "fisher_p": float(stats.chi2.sf(chi, 2 * len(u))),
            "mean": float(np.mean(u)), "below_0.2": int(np.sum(u < 0.2))}
