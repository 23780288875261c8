"""Convert the reference's ``codes_lib`` parity-check data into bundled CSR ``.npz``.

Run in the build container (``/root/reference`` is absent on the GPU box):

    python tools/import_codes.py [/root/reference/codes_lib]

Inputs are data files only: ``hgp_34_n225.pkl`` is read by the non-executing
opcode reader (:mod:`qldpc_fault_tolerance_amd.safepickle`), ``.mat`` by
``scipy.io.loadmat``, ``.npy`` by ``numpy.load(allow_pickle=False)``.  Logicals of
the ``.mat``/``.npy`` codes are computed as ``bposd.css.css_code`` does
(:func:`gf2.compute_logicals`).  The missing HGP codes are synthesised by
``tools/synth_hgp_codes.py``.
"""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from qldpc_fault_tolerance_amd import codes  # noqa: E402

SRC = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/codes_lib"

JOBS = [
    ("hgp_34_n225", "hgp_34_n225.pkl", None),
    ("GenBicycleA1", "GenBicycleA1_hx.mat", "GenBicycleA1_hz.mat"),
    ("GenBicycleA2", "GenBicycleA2_hx.mat", "GenBicycleA2_hz.mat"),
    ("GenBicycleA3", "GenBicycleA3_hx.mat", "GenBicycleA3_hz.mat"),
    ("GenBicycleA4", "GenBicycleA4_hx.mat", "GenBicycleA4_hz.mat"),
    ("LP_Matg8_L16_Dmin12", "LP_Matg8_L16_Dmin12_hx.mat", "LP_Matg8_L16_Dmin12_hz.mat"),
    ("LP_Matg8_L21_Dmin16", "LP_Matg8_L21_Dmin16_hx.mat", "LP_Matg8_L21_Dmin16_hz.mat"),
    ("LP_Matg8_L30_Dmin20", "LP_Matg8_L30_Dmin20_hx.mat", "LP_Matg8_L30_Dmin20_hz.mat"),
    ("tanner_code1", "tanner_code1_hx.npy", "tanner_code1_hz.npy"),
]


def main():
    os.makedirs(codes.CODES_LIB, exist_ok=True)
    for name, fx, fz in JOBS:
        px = os.path.join(SRC, fx)
        pz = os.path.join(SRC, fz) if fz else None
        code = codes.load_code(px, pz, name=name)
        code.name = name
        assert code.test(), name
        codes.save_npz(code, os.path.join(codes.CODES_LIB, name + ".npz"))
        print(f"{name}: [[{code.N},{code.K}]] hx {code.hx.shape} hz {code.hz.shape}")


if __name__ == "__main__":
    main()
