"""Which engine / kernel family serves each bundled code's graphs (diagnostic; round 6).

    python tools/route_survey.py [precision]

For every bundled code: hz itself and GetSpaceTimeCheckMat(hz, t0) for t0 = 2..5 (the phenomenological
space-time decoders of CodeFamily_SpaceTime.EvalWER('phenl', num_rep = t0)), and [hz | I] (the
single-shot CodeSimulator_Phenon decoder1): one JSON line with the shape, the row / column degrees and
the decoder's geometry.  QLDPC_M2S_ANNEAL=0 skips the placement search (routing does not depend on it).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("QLDPC_M2S_ANNEAL", "0")
import numpy as np  # noqa: E402

from qldpc_fault_tolerance_amd import codes  # noqa: E402
from qldpc_fault_tolerance_amd.engine import DeviceBP  # noqa: E402

prec = int(sys.argv[1]) if len(sys.argv) > 1 else 64
for name in codes.bundled_codes():
    code = codes.get_code(name)
    hz = code.hz
    m, n = hz.shape
    graphs = [("hz", codes.CSR.from_dense(hz))] + [(f"st{t0}", codes.space_time_csr(hz, t0)) for t0 in range(2, 6)]
    graphs.append(("hI", codes.CSR.from_dense(np.hstack([hz, np.eye(m, dtype=np.uint8)]))))
    for tag, H in graphs:
        deg = np.bincount(H.col_idx, minlength=H.n)
        rec = {"code": name, "graph": tag, "m": H.m, "n": H.n, "nnz": int(len(H.col_idx)),
               "max_row": int(np.diff(H.row_ptr).max()), "max_col": int(deg.max())}
        try:
            g = DeviceBP(H, 0.01 * np.ones(H.n), max_iter=10, precision=prec).geometry()
            rec.update({k: g[k] for k in ("engine", "kernel_id", "threads", "vars_per_thread", "lds_bytes", "blocks_per_cu")})
        except Exception as e:  # noqa: BLE001
            rec["error"] = repr(e)[:200]
        print(json.dumps(rec), flush=True)
