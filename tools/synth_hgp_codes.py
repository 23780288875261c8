"""Synthesise stand-ins for the reference's missing HGP pickles.

``codes_lib/hgp_34_n1600.pkl`` and ``hgp_34_n1225_q3.pkl`` (and the n625 ones)
are listed in the reference's ``.MISSING_LARGE_BLOBS``.  They were made by
``QuantumExpanderFromCheckMat`` = ``hgp(H, H)`` of a random (Δc=4, Δv=3) Tanner
graph from ``RandomaGraphs(n0, 4, 3)`` (``src/QuantumExanderCodesGene.py:30-34,
181-233``): n0=8 → 24×32 → [[1600,64]], n0=7 → 21×28 → [[1225,49]], n0=5 → 15×20
→ [[625,25]].  The exact instances are lost, so this script rebuilds instances
with the same parameters (N, K, degrees) from a fixed seed; the seed and the
resulting check matrix are committed (``codes_lib/*.npz``).

    python tools/synth_hgp_codes.py
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from qldpc_fault_tolerance_amd import codes  # noqa: E402

SEED = 0x51D5EED0
JOBS = [
    # name, n0, expected K (Threshold-checkpoint.ipynb:233-236), girth target
    ("hgp_34_n625", 5, 25, 6),
    ("hgp_34_n1225_q3", 7, 49, 6),
    ("hgp_34_n1600", 8, 64, 6),
]


def main():
    os.makedirs(codes.CODES_LIB, exist_ok=True)
    for name, n0, K, girth in JOBS:
        h = codes.random_biregular_check_matrix(n0, 4, 3, seed=SEED + n0, min_girth=girth)
        code = codes.hgp(h, h, name=name)
        assert code.K == K, (name, code.K)
        assert code.test(), name
        codes.save_npz(code, os.path.join(codes.CODES_LIB, name + ".npz"))
        print(f"{name}: h {h.shape} girth {codes.tanner_girth(h)} -> [[{code.N},{code.K}]] "
              f"hx {code.hx.shape} E={int(code.hx.sum())}")


if __name__ == "__main__":
    main()
