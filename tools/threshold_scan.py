"""GPU threshold scan of the synthetic (3,4) HGP family under the headline decoder.

Picks bench.py's operating point: the code-capacity ``EvalWER('data')`` sweep
(src/Simulators.py:759-777) of hgp_34_n225 / n625 / n1600 with min-sum
alpha=0.625, max_iter=int(N/10), eval_logical_type='Total'.  Prints one JSON
line per (code, p) with LER, WER (A8 formula), mean iterations and the
non-converged fraction.

    python tools/threshold_scan.py [shots]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from qldpc_fault_tolerance_amd import codes  # noqa: E402
from qldpc_fault_tolerance_amd.engine import DeviceBP, DeviceMC  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
P = [0.02, 0.03, 0.04, 0.05, 0.06, 0.07, 0.08, 0.10, 0.12]
for name in ("hgp_34_n225", "hgp_34_n625", "hgp_34_n1600"):
    code = codes.get_code(name)
    n = code.N
    mi = int(n / 10)
    for ep in P:
        pp = ep * 3 / 2 / 3
        dx = DeviceBP(code.hz, ep * np.ones(n), max_iter=mi, precision=32)
        dz = DeviceBP(code.hx, ep * np.ones(n), max_iter=mi, precision=32,
                      vars_per_thread=dx.geometry()["vars_per_thread"])
        mc = DeviceMC(code, dx, dz)
        t0 = time.perf_counter()
        r = mc.run(pp, pp, pp, seed=7, shot_begin=0, shot_count=S, logical_mode="Total")
        dt = time.perf_counter() - t0
        ler = r.failures / r.shots
        wer = 1.0 - (1 - ler) ** (1 / code.K)
        dec = sum(r.sector_decodes)
        print(json.dumps({"code": name, "p": ep, "shots": r.shots, "ler": ler, "wer": wer,
                          "iters": sum(r.sector_iters) / dec, "nonconv": sum(r.sector_nonconv) / dec,
                          "shots_per_s": r.shots / dt}), flush=True)
