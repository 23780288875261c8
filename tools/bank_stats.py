"""Print engine-3 geometry and gather bank-conflict stats (before/after check labelling) per code/precision."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from qldpc_fault_tolerance_amd import codes  # noqa: E402
from qldpc_fault_tolerance_amd.engine import DeviceBP  # noqa: E402

for name in (sys.argv[1:] or ["hgp_34_n1600", "hgp_34_n225", "LP_Matg8_L30_Dmin20", "GenBicycleA4"]):
    code = codes.get_code(name)
    for prec in (64, 32):
        t0 = time.perf_counter()
        d = DeviceBP(code.hz, 0.05 * np.ones(code.N), max_iter=10, precision=prec)
        dt = time.perf_counter() - t0
        print(name, prec, d.geometry(), f"create {dt * 1e3:.0f} ms", flush=True)
