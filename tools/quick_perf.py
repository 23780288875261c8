"""Quick throughput probe of the fused MC kernel (dev tool)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from qldpc_fault_tolerance_amd import codes
from qldpc_fault_tolerance_amd.engine import DeviceBP, DeviceMC

name = sys.argv[1] if len(sys.argv) > 1 else "hgp_34_n1600"
code = codes.get_code(name)
n = code.N
for prec in (32, 64):
    for vpl in [0] + [int(x) for x in os.environ.get("VPLS", "").split(",") if x]:
        for p in (0.02, 0.04, 0.06):
            dx = DeviceBP(code.hz, p * np.ones(n), max_iter=int(n / 10), precision=prec, vars_per_thread=vpl)
            mc = DeviceMC(code, dx, None)
            g = dx.geometry()
            S = 1 << 16
            cnt = mc.new_counters()
            mc.launch(p/2, p/2, p/2, 1, 0, 4096, "X", cnt)
            torch.cuda.synchronize()
            cnt.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            mc.launch(p/2, p/2, p/2, 1, 0, S, "X", cnt)
            e1.record(); torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            w = cnt.cpu().numpy()
            its = w[4] / w[0]
            E = int(code.hz.sum())
            print(f"{name} fp{prec} vpl={g['vars_per_thread']} TB={g['threads']} bpc={g['blocks_per_cu']} p={p}: "
                  f"{S/ms*1e3:,.0f} shots/s  iters/shot={its:.1f}  LER={w[1]/w[0]:.4f}  "
                  f"edge-iters/s={S*its*E/ms*1e3:.3e}", flush=True)
