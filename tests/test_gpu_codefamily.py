"""GPU-backed CodeFamily sweeps (src/Simulators.py:746-809,
src/Simulators_SpaceTime.py:1152-1217) against the oracle's counts on n225.

Every simulator an EvalWER sweep builds draws its Philox seed from CPython's ``random`` at its
first batch (``random.getrandbits(64)``), so seeding ``random`` before the sweep fixes every
(code, p) stream; the oracle then runs the same streams and the reference's WER formulas are
applied to its counts.
"""
import random

import numpy as np
import pytest

from qldpc_fault_tolerance_amd import codes, decoders, simulators

pytestmark = pytest.mark.gpu


def _classes():
    bp = decoders.BP_Decoder_Class(max_iter_ratio=10, bp_method="minimum_sum", ms_scaling_factor=0.625)
    st = decoders.ST_BP_Decoder_Class(max_iter_ratio=10, bp_method="minimum_sum", ms_scaling_factor=0.625)
    return bp, st


def test_codefamily_evalwer_data(gpu, oracle):
    code = codes.get_code("hgp_34_n225")
    bp, _ = _classes()
    p_list, S = [0.03, 0.06], 2000
    random.seed(77)
    wer = simulators.CodeFamily([code], bp, bp).EvalWER("data", "Total", p_list, S, if_plot=False)
    random.seed(77)
    want = []
    for p in p_list:
        seed = random.getrandbits(64)
        r = oracle.mc_run(code, p / 2, p / 2, p / 2, seed=seed, shot_begin=0, shot_count=S, logical_mode="Total",
                          probs_x=p, probs_z=p, max_iter=22, precision=64)
        want.append(simulators.word_error_rate(r["failures"], S, code.K)[0])
    assert wer.shape == (1, 2)
    assert wer[0].tolist() == want


def test_codefamily_evalwer_phenl(gpu, oracle):
    """'phenl' branch: CodeSimulator_Phenon (num_rep = 1) with decoder1 on [h | I] (p_syndrome) and decoder2 on h."""
    code = codes.get_code("hgp_34_n225")
    bp, _ = _classes()
    p_list, S, cycles = [0.01, 0.02], 800, 3
    random.seed(5)
    wer = simulators.CodeFamily([code], bp, bp).EvalWER("phenl", "Total", p_list, S, num_cycles=cycles, if_plot=False)
    random.seed(5)
    want = []
    for p in p_list:
        seed = random.getrandbits(64)
        pd = p * 3 / 2 * 2 / 3
        r = oracle.phenl_run(code, p / 2, p / 2, p / 2, p, seed, 0, S, cycles, 1, "Total", p_data=pd, p_synd=p)
        want.append(simulators.word_error_rate_phenl(r["failures"], S, code.K, cycles))
    assert wer[0].tolist() == want


def test_codefamily_spacetime_evalwer(gpu, oracle):
    """CodeFamily_SpaceTime.EvalWER: 'data' and 'phenl' (num_rep 3); returns (per-code WER arrays, p grids)."""
    code = codes.get_code("hgp_34_n225")
    bp, st = _classes()
    fam = simulators.CodeFamily_SpaceTime([code], st, bp)
    p_list, S = [0.01, 0.02], 600
    random.seed(9)
    wl, pl = fam.EvalWER("phenl", "Total", p_list, S, num_cycles=7, num_rep=3, if_plot=False)
    random.seed(9)
    want = []
    for p in p_list:
        seed = random.getrandbits(64)
        r = oracle.phenl_run(code, p / 2, p / 2, p / 2, p, seed, 0, S, 3, 3, "Total", p_data=p, p_synd=p)
        want.append(simulators.word_error_rate_per_cycle(r["failures"], S, code.K, 7))
    assert len(wl) == 1 and wl[0].tolist() == want and pl[0].tolist() == p_list
    random.seed(10)
    wl, pl = fam.EvalWER("data", "X", [0.05], S, if_plot=False)
    assert pl == [0.05]  # the p list as passed (src/Simulators_SpaceTime.py:1166)
    random.seed(10)
    seed = random.getrandbits(64)
    r = oracle.mc_run(code, 0.025, 0.025, 0.025, seed=seed, shot_begin=0, shot_count=S, logical_mode="X",
                      probs_x=0.05, probs_z=0.05, max_iter=22, precision=64)
    assert wl[0].tolist() == [simulators.word_error_rate(r["failures"], S, code.K)[0]]
