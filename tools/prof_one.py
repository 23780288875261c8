"""One fused MC launch (for rocprofv3 --pmc passes): python tools/prof_one.py [code] [p] [shots] [vpl] [precision]."""
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
code = codes.get_code(name)
n = code.N
dx = DeviceBP(code.hz, p * np.ones(n), max_iter=int(n / 10), precision=prec, vars_per_thread=vpl)
mc = DeviceMC(code, dx, None)
cnt = mc.new_counters()
pp = p * 3 / 2 / 3
mc.launch(pp, pp, pp, 1, 0, S, "X", cnt)
torch.cuda.synchronize()
w = cnt.cpu().numpy()
print(f"{name} p={p} shots={S} geometry={dx.geometry()} iters/decode={w[4] / w[0]:.1f}")
