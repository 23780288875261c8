"""One fused MC launch of the bench workload (for rocprofv3 --pmc passes):

    python tools/prof_one.py [code] [p] [shots] [vpl] [precision] [logical] [seed] [max_iter_ratio]

Builds the decoders exactly as bench.py's data workload does (p_data = eval_p on hz and hx,
min-sum alpha 0.625, max_iter = int(N / ratio), the Z sector taking the X sector's geometry) and
issues ONE launch of ``shots`` shots with Pauli probabilities [p/2]*3.  logical "X" (the default
of older callers) launches the X sector only.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from qldpc_fault_tolerance_amd import codes  # noqa: E402
from qldpc_fault_tolerance_amd.engine import DeviceBP, DeviceMC  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "hgp_34_n1600"
p = float(sys.argv[2]) if len(sys.argv) > 2 else 0.06
S = int(sys.argv[3]) if len(sys.argv) > 3 else 8192
vpl = int(sys.argv[4]) if len(sys.argv) > 4 else 0
prec = int(sys.argv[5]) if len(sys.argv) > 5 else 32
logical = sys.argv[6] if len(sys.argv) > 6 else "X"
seed = int(sys.argv[7]) if len(sys.argv) > 7 else 1
ratio = float(sys.argv[8]) if len(sys.argv) > 8 else 10.0
code = codes.get_code(name)
n = code.N
mi = int(n / ratio)
dx = DeviceBP(code.hz, p * np.ones(n), max_iter=mi, precision=prec, vars_per_thread=vpl) if logical != "Z" else None
v2 = dx.geometry()["vars_per_thread"] if dx is not None and not os.environ.get("QLDPC_TB") else vpl
dz = DeviceBP(code.hx, p * np.ones(n), max_iter=mi, precision=prec, vars_per_thread=v2) if logical != "X" else None
mc = DeviceMC(code, dx, dz)
cnt = mc.new_counters()
pp = p * 3 / 2 / 3
mc.launch(pp, pp, pp, seed, 0, S, logical, cnt)
torch.cuda.synchronize()
w = cnt.cpu().numpy()
dec = max(1, int(w[2] + w[3]))
print(f"{name} p={p} shots={S} logical={logical} precision={prec} geometry={(dx or dz).geometry()} "
      f"decodes={dec} iters/decode={(w[4] + w[5]) / dec:.3f}")
