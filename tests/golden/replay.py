"""Helpers for replaying the reference-harness fixtures (tests/golden/make_golden.py).

The fixtures record CPython ``random`` seeds rather than the uniforms themselves: re-seeding
``random`` and drawing ``random.random()`` regenerates exactly the stream the reference's
``_generate_error`` consumed (MT19937, 53-bit doubles), here and on the GPU box.
"""
import os
import random

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
CONFIGS = os.path.join(HERE, "reference_harness_configs.npz")
CONFIG_CODES = ["hgp_34_n1600", "LP_Matg8_L30_Dmin20", "GenBicycleA1", "GenBicycleA2", "GenBicycleA3", "GenBicycleA4"]


def uniforms(seed0: int, count: int, per_shot: int) -> np.ndarray:
    """[count, per_shot] uniforms: shot s draws after random.seed(seed0 + s)."""
    state = random.getstate()
    try:
        out = np.empty((count, per_shot))
        for s in range(count):
            random.seed(seed0 + s)
            out[s] = [random.random() for _ in range(per_shot)]
        return out
    finally:
        random.setstate(state)


def unpack(a: np.ndarray, width: int) -> np.ndarray:
    return np.unpackbits(a, axis=-1)[..., :width]
