"""Pin of the BP / BP+OSD arithmetic against fits the reference printed with the REAL ldpc/bposd.

The only outputs in the reference that the third-party ``ldpc.bp_decoder`` and
``bposd.bposd_decoder`` produced are the threshold fits printed by
``.ipynb_checkpoints/Threshold-checkpoint.ipynb`` (cells 16, 20, 25: phenomenological noise on
the LP [[544,80]]/[[714,100]]/[[1020,136]] family and on the d5/d9/d13 toric codes; values and
notebook line numbers in ``tests/notebook_pin.py:PRINTED``).  Each point is the notebook's
``CodeFamilyPhenlThreshold`` (lines 127-170) on this engine: ``CodeSimulator_Phenon``,
decoder1 = ``BPDecoder`` on ``[h | I]`` (``int(N/30)`` iterations), decoder2 = ``BPOSD_Decoder``
OSD-E(10) (``int(N/10)``), fused on the GPU, with the syndrome-flip rate of the adopted
per-cell hypothesis (``notebook_pin.ADOPTED``: q = 2p/3 for the LP cells, q = 0 for the toric
cell, which the notebook ran before the definition the LP cells used; the hypothesis table of
round 4 is ``profiles/r04/pin/hypotheses.json``).

The engine's failure probabilities (25x the notebook's samples) define the distribution of the
notebook's experiment under "same decoder statistics"; a parametric bootstrap (binomial counts at
the notebook's sample sizes, refit with the notebook's own ``ThresholdEst``) places every printed
(A, p_c) at a percentile of that distribution.  Under the null the 15 percentiles are U(0, 1):
the criterion is a combined uniformity test (KS and Fisher's method), which replaces round 3's
"at most 2 of 15 outside the 95 % bands" (that criterion passed at q = 0 with KS p = 0.006).
"""
import numpy as np
import pytest

import notebook_pin as nbp

pytestmark = pytest.mark.gpu

MULT = 25
DRAWS = 400


@pytest.fixture(scope="module")
def engine_counts(gpu):
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from notebook_pin_run import cell_counts

    return {cell: cell_counts(cell, MULT, 0x5EED, 64, log=lambda s: None, hyp=nbp.ADOPTED[cell]) for cell in (16, 20, 25)}


@pytest.fixture(scope="module")
def heldout_counts(gpu):
    """A fresh 25x sample under the ADOPTED hypotheses at notebook_pin.HELDOUT_SEED (round 5)."""
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from notebook_pin_run import cell_counts

    return {cell: cell_counts(cell, MULT, nbp.HELDOUT_SEED, 64, log=lambda s: None, hyp=nbp.ADOPTED[cell])
            for cell in (16, 20, 25)}


def _pct(cell, counts, formula="current"):
    """Mid-rank percentile of each printed (A, p_c) in the bootstrap distribution, plus the bands."""
    P = nbp.cell_p_list(cell)
    out = {}
    for R, c in counts.items():
        fp = np.asarray(c["fail"], dtype=np.float64) / c["samples"]
        b = nbp.bootstrap_band(fp, c["K"], P, nbp.cell_samples(cell, R), R, formula=formula, draws=DRAWS,
                               seed=17 + R + cell)
        A0, pc0, line = nbp.PRINTED[cell][R]
        out[R] = {"A_pct": nbp.mid_percentile(A0, b["fits"][:, 0]), "p_c_pct": nbp.mid_percentile(pc0, b["fits"][:, 1]),
                  "line": line, "failed": b["failed"], "fail_prob": fp}
    return out


def test_printed_fits_uniform_in_engine_distribution(engine_counts):
    res = {cell: _pct(cell, engine_counts[cell]) for cell in (16, 20, 25)}
    pts = [(cell, R, e) for cell, d in res.items() for R, e in d.items()]
    assert len(pts) == 15
    pc = nbp.uniformity([e["p_c_pct"] for _, _, e in pts])
    A = nbp.uniformity([e["A_pct"] for _, _, e in pts])
    print("p_c percentiles:", [(cell, R, round(e["p_c_pct"], 3)) for cell, R, e in pts])
    print("p_c uniformity:", pc, "A uniformity:", A)
    # round 4 measured (profiles/r04/pin/): p_c KS p = 0.51, Fisher p = 0.105; A KS p = 0.18.  ADOPTED
    # was selected on THIS seed from 36 hypothesis combinations: the Bonferroni-corrected values are
    # the honest ones for this run (the held-out seed below carries the pre-registered test)
    print("Bonferroni x", nbp.HYPOTHESIS_COMBINATIONS, ": p_c KS", nbp.bonferroni(pc["ks_p"]), "Fisher",
          nbp.bonferroni(pc["fisher_p"]), "; A KS", nbp.bonferroni(A["ks_p"]), "Fisher", nbp.bonferroni(A["fisher_p"]))
    assert pc["ks_p"] > 0.05 and pc["fisher_p"] > 0.05, pc
    assert A["ks_p"] > 0.05, A
    # fits that failed inside the bootstrap stay rare (the notebook's fit itself succeeded every time)
    assert all(e["failed"] <= DRAWS // 20 for _, _, e in pts)


def test_heldout_seed_uniform(heldout_counts):
    """The pre-registered check: the ADOPTED hypotheses on a fresh 25x sample
    (notebook_pin.HELDOUT_SEED, never used for selection).  p_c: KS and Fisher p > 0.05; A: KS p > 0.05.
    A's Fisher test is reported, not asserted: it fails at BOTH seeds (selection 0.012, held-out 0.013,
    profiles/r05/pin/summary.json), so it is a reproducible residual, not a selection artefact: the
    printed amplitudes sit low in the engine's distribution (mean percentile 0.38-0.39, 6-7 of 15 below
    0.2) while KS does not reject (0.18 / 0.25).  A is the fit's amplitude, jointly fitted with p_c; the
    adopted hypotheses explain p_c (KS 0.90 held out) but leave this A offset unexplained; recorded."""
    res = {cell: _pct(cell, heldout_counts[cell]) for cell in (16, 20, 25)}
    pts = [(cell, R, e) for cell, d in res.items() for R, e in d.items()]
    assert len(pts) == 15
    pc = nbp.uniformity([e["p_c_pct"] for _, _, e in pts])
    A = nbp.uniformity([e["A_pct"] for _, _, e in pts])
    print("held-out seed", hex(nbp.HELDOUT_SEED), "p_c percentiles:", [(cell, R, round(e["p_c_pct"], 3)) for cell, R, e in pts])
    print("held-out p_c uniformity:", pc, "A uniformity:", A)
    assert pc["ks_p"] > 0.05 and pc["fisher_p"] > 0.05, pc
    assert A["ks_p"] > 0.05, A


def test_fit_at_engine_rates_tracks_printed(engine_counts):
    """The best-conditioned fits (rounds 6-20, where every code's rate is far from 0 and 1): the
    notebook's ThresholdEst applied to the engine's own rates reproduces the printed p_c within 15 %
    (measured: LP 0.3-7.2 %, toric 0.04-13.4 %)."""
    for cell in (16, 20, 25):
        P = nbp.cell_p_list(cell)
        for R, c in engine_counts[cell].items():
            if R > 20:
                continue
            fp = np.asarray(c["fail"], dtype=np.float64) / c["samples"]
            wer = np.vstack([nbp.wer_current(fp[i] * c["samples"], c["samples"], c["K"][i], R) for i in range(3)])
            _, pc = nbp.threshold_est(P, wer)
            pc0 = nbp.PRINTED[cell][R][1]
            assert abs(pc - pc0) / pc0 < 0.15, (cell, R, pc, pc0)


def test_commented_wer_transform_ruled_out(engine_counts):
    """At 30 rounds the engine's toric d13 failure rate at p = 0.02 exceeds 0.5, where the
    commented-out transform (src/Simulators.py:343) is NaN and curve_fit raises: the printed
    30-round fit (notebook line 900) was made with the current transform."""
    c = engine_counts[25][30]
    fp = np.asarray(c["fail"], dtype=np.float64) / c["samples"]
    assert fp[2, -1] > 0.5
    wer = np.vstack([nbp.wer_commented(fp[i] * c["samples"], c["samples"], c["K"][i], 30) for i in range(3)])
    assert not np.all(np.isfinite(wer))
