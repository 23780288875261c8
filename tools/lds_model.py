"""Static LDS model of the headline decoders vs the measured bank-conflict share.

    python tools/lds_model.py [code] [p]      (GPU box: building a decoder needs the device)

Prints, per sector, qldpc_bp_lds_model's per-workgroup-iteration cycles of the variable phase
(CS gathers, V-slot reads, v2c stores: LDS-array cycles and the bank-conflict extra) and the
conflict-free check phase of the m2s kernel (rows as 3 x ds_read_b128 + the tail ds_read_b64,
the F word, CS + argmin ds_write_b64: 24 cycles per wave-row pass), so the modelled conflict share
can be set against SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from qldpc_fault_tolerance_amd import codes  # noqa: E402
from qldpc_fault_tolerance_amd.engine import DeviceBP  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "hgp_34_n1600"
p = float(sys.argv[2]) if len(sys.argv) > 2 else 0.06
code = codes.get_code(name)
out = {}
for sec, H in (("hz", code.hz), ("hx", code.hx)):
    d = DeviceBP(H, p * np.ones(code.N), max_iter=int(code.N / 10), precision=64)
    g = d.geometry()
    lm = g["lds_model"]
    m = H.shape[0]
    waves = g["threads"] // 64
    passes = -(-m // g["threads"])
    check = 24 * passes * waves if g["kernel_id"] == 11103 else None
    var = lm["cs_gather"] + lm["v_read"] + lm["v_store"]  # one LDS-array cycle per conflict-free lane group
    extra = lm["cs_gather_extra"] + lm["v_read_extra"] + lm["v_store_extra"]
    out[sec] = {"geometry": {k: g[k] for k in ("kernel_id", "threads", "vars_per_thread", "degree3_slots")},
                "lds_model": lm, "var_phase_array_cycles": var, "var_phase_extra": extra,
                "check_phase_cycles": check,
                "modelled_conflict_share": extra / (var + (check or 0)) if check else None}
print(json.dumps(out, indent=1))
