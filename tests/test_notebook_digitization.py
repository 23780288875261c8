"""CPU checks on ``tests/golden/notebook_plot_points.json``: the data points read off the Threshold
notebook's fit plots by ``tools/notebook_digitize.py`` (the notebook's embedded PNG outputs of
``ThresholdEst(if_plot=True)``, reference .ipynb_checkpoints/Threshold-checkpoint.ipynb lines 71-120).

The fixture backs DESIGN.md §2's per-point comparison of the notebook with the engine.  These tests pin
what makes it trustworthy: the axes calibrate to sub-pixel residuals, the pixels map back to the stored
WER through the stored calibration, and the fit of the digitized points reproduces the (A, p_c) the
notebook printed for every plot whose markers are all legible.  Three plots are recorded as not pinned
(listed below, with the reason) and are excluded from the analysis as well as from these bounds."""
import math
import os
import json

import numpy as np
import pytest

import notebook_pin as nbp

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = json.load(open(os.path.join(HERE, "golden", "notebook_plot_points.json")))

# (cell, rounds): cell 16 R25/R30 have 6 and 3 of their markers hidden under later colours (the refit
# misses the printed p_c by 16%/15%); cell 25 R6 has equally spaced ticks without log sub-ticks, so its
# decades-per-tick scale is not read from the plot
NOT_PINNED = {(16, 25), (16, 30), (25, 6)}


def _plots():
    return [pytest.param(p, id=f"cell{p['cell']}_R{p['rounds']}") for p in FIX["plots"]]


def test_fixture_covers_the_three_cells():
    cells = sorted({p["cell"] for p in FIX["plots"]})
    assert cells == [16, 20, 25]
    assert len(FIX["plots"]) == 15


@pytest.mark.parametrize("plot", _plots())
def test_axes_calibrate_to_subpixel(plot):
    assert plot["y_axis"]["tick_rms_px"] < 0.5
    assert plot["x_rms_px"] < 0.5
    assert plot["y_axis"]["b_px_per_decade"] < 0  # image rows grow downwards


@pytest.mark.parametrize("plot", _plots())
def test_pixels_map_to_stored_wer(plot):
    ya = plot["y_axis"]
    for row_px, row_w in zip(plot["pixels"], plot["wer"]):
        for (_, y), w in zip(row_px, row_w):
            logv = (y - ya["a"]) / ya["b_px_per_decade"] + ya["decade"]
            # pixels are stored to 0.01 px: 0.01 / 111 px-per-decade ~ 1e-4 decades
            assert math.isclose(10.0 ** logv - 1e-6, w, rel_tol=2e-3, abs_tol=1e-12)


@pytest.mark.parametrize("plot", _plots())
def test_refit_reproduces_printed_fit(plot):
    A, pc = nbp.threshold_est(np.array(plot["p"]), np.array(plot["wer"]))
    assert math.isclose(A, plot["refit"]["A"], rel_tol=1e-6)
    assert math.isclose(pc, plot["refit"]["p_c"], rel_tol=1e-6)
    if (plot["cell"], plot["rounds"]) in NOT_PINNED:
        pytest.skip("recorded as not pinned (see NOT_PINNED)")
    assert abs(pc / plot["printed"]["p_c"] - 1) < 0.06
    assert abs(A / plot["printed"]["A"] - 1) < 0.20
