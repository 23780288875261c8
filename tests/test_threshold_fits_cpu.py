"""Threshold tooling against the reference's own fit functions.

tests/golden/reference_fits.npz was produced by running the reference's DistanceEst,
ThresholdEst_extrapolation and CodeFamily{,_SpaceTime}.EvalThreshold / EvalSustainableThreshold /
EvalEffectiveDistances (src/Simulators.py:675-741, 912-963; src/Simulators_SpaceTime.py:1080-1149,
1311-1362) on fixed injected WER arrays, with EvalWER / EvalThreshold replaced by recorders.
"""
import os

import numpy as np
import pytest

from qldpc_fault_tolerance_amd import simulators

FITS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_fits.npz")


@pytest.fixture(scope="module")
def g():
    return np.load(FITS, allow_pickle=False)


def test_distance_and_threshold_extrapolation(g):
    np.testing.assert_allclose(simulators.DistanceEst(g["thr_p"], g["thr_wer"]), g["sim_distance_est"], rtol=1e-9)
    np.testing.assert_allclose(simulators.ThresholdEst_extrapolation(g["thr_p"], g["thr_wer"]),
                               g["sim_threshold_extrap"][0], rtol=1e-9)


def _recording(data, seen):
    def f(self, noise_model, eval_logical_type, eval_p_list, *a, **k):
        seen.append(np.array(eval_p_list, dtype=np.float64))
        return data
    return f


@pytest.mark.parametrize("cls", [simulators.CodeFamily, simulators.CodeFamily_SpaceTime])
def test_eval_threshold_and_effective_distances(g, monkeypatch, cls):
    seen = []
    st = cls is simulators.CodeFamily_SpaceTime
    fam = cls([], None, None)
    monkeypatch.setattr(cls, "EvalWER", _recording((list(g["thr_wer"]), None) if st else g["thr_wer"], seen))
    np.testing.assert_allclose(fam.EvalThreshold("data", "Total", "extrapolation", 0.08, 100),
                               g["fam_eval_threshold"][0], rtol=1e-9)
    np.testing.assert_allclose(seen[-1], g["fam_eval_threshold_p"], rtol=0, atol=0)
    monkeypatch.setattr(cls, "EvalWER", _recording((list(g["dist_wer"]), None) if st else g["dist_wer"], seen))
    want = g["st_eval_distances"] if st else g["fam_eval_distances"]
    np.testing.assert_allclose(fam.EvalEffectiveDistances("data", "Total", "extrapolation", 0.08, 100), want, rtol=1e-9)
    np.testing.assert_allclose(seen[-1], g["st_eval_distances_p" if st else "fam_eval_distances_p"], rtol=0, atol=0)


@pytest.mark.parametrize("cls,key", [(simulators.CodeFamily, "fam"), (simulators.CodeFamily_SpaceTime, "st")])
def test_sustainable_threshold(g, monkeypatch, cls, key):
    cycles, thr = list(g["sus_cycles"]), g["sus_thr"]
    calls = []

    def rec(self, noise_model, eval_logical_type, eval_method, est_threshold, num_samples, num_cycles=1, **k):
        calls.append([num_samples, num_cycles])
        return float(thr[cycles.index(num_cycles)])

    monkeypatch.setattr(cls, "EvalThreshold", rec)
    p_sus = cls([], None, None).EvalSustainableThreshold("phenl", "Total", "extrapolation", 0.05, 12000, cycles)
    np.testing.assert_allclose(p_sus, g[f"{key}_sus"][0], rtol=1e-9)
    assert calls == g[f"{key}_sus_calls"].tolist()


def test_notebook_threshold_est_restatement_matches_notebook():
    """tests/notebook_pin.threshold_est == the Threshold notebook's own ThresholdEst (cells 1-2,
    executed from the notebook source by tests/golden/make_golden.py notebook) on 18 WER arrays."""
    import os

    import notebook_pin as nbp

    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "notebook_fits.npz"),
                allow_pickle=False)
    for k in range(int(g["ncases"][0])):
        A, pc = g[f"case{k}_A_pc"]
        got = nbp.threshold_est(g[f"case{k}_p"], g[f"case{k}_wer"])
        assert np.isclose(got[0], A, rtol=1e-9, atol=0) and np.isclose(got[1], pc, rtol=1e-9, atol=0), (k, got, A, pc)


def test_notebook_pin_wer_transforms():
    """The two WER transforms of CodeSimulator_Phenon.WordErrorRate (src/Simulators.py:341-351,
    commented; :353-360, current) agree with each other for small rates, and the current one
    equals the drop-in's word_error_rate_phenl at odd round counts."""
    import notebook_pin as nbp
    from qldpc_fault_tolerance_amd.simulators import word_error_rate_phenl

    for c, S, K, R in ((3, 1000, 80, 5), (40, 400, 136, 9), (0, 500, 2, 7), (300, 600, 2, 3)):
        assert np.isclose(nbp.wer_current(c, S, K, R), word_error_rate_phenl(c, S, K, R), rtol=1e-12, atol=0)
    a, b = nbp.wer_commented(1, 10000, 100, 6), nbp.wer_current(1, 10000, 100, 6)
    assert np.isclose(a, b, rtol=1e-3)


def test_pin_uniformity_statistics():
    """tests/notebook_pin.py's combined test: mid-rank percentiles never hit 0
    or 1, uniform percentiles pass, percentiles crowded at one end fail both KS and Fisher."""
    import notebook_pin as nbp

    fits = np.linspace(0.0, 1.0, 101)
    assert 0 < nbp.mid_percentile(-1.0, fits) < 0.01 and 0.99 < nbp.mid_percentile(2.0, fits) < 1
    assert abs(nbp.mid_percentile(0.5, fits) - 0.5) < 1e-9
    u = nbp.uniformity((np.arange(15) + 0.5) / 15)
    assert u["ks_p"] > 0.9 and u["fisher_p"] > 0.5
    low = nbp.uniformity(np.full(15, 0.03))
    assert low["ks_p"] < 1e-6 and low["fisher_p"] < 1e-6
