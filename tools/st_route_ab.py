"""Time one fp64 space-time decode_batch on a given code / round count (round-6 routing A/B).

    QLDPC_E3_TAIL=0|1 python tools/st_route_ab.py [code] [t0] [p] [syndromes]     (t0 = 0: hz itself)

Builds the hz space-time decoder as bench.py --workload phenl does (min-sum alpha 0.625, max_iter
int(n/10), fp64), decodes i.i.d.-error syndromes generated on the GPU, one warm-up launch then three
timed launches (HIP events on torch's stream), and prints the geometry, ms per launch and mean iterations.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from qldpc_fault_tolerance_amd import codes  # noqa: E402
from qldpc_fault_tolerance_amd.engine import DeviceBP  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "hgp_34_n1600"
t0 = int(sys.argv[2]) if len(sys.argv) > 2 else 2
p = float(sys.argv[3]) if len(sys.argv) > 3 else 0.01
B = int(sys.argv[4]) if len(sys.argv) > 4 else 32768
code = codes.get_code(name)
n = code.N
# t0 = 0: hz itself (the data-error / BP+OSD decoders)
Hst = codes.space_time_csr(code.hz, t0) if t0 > 0 else codes.CSR.from_dense(code.hz)
probs = np.hstack([p * np.ones(n), p * np.ones(code.hz.shape[0])] * t0) if t0 > 0 else p * np.ones(n)
dec = DeviceBP(Hst, probs, max_iter=int(n / 10), precision=64)
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(7)
Hd = torch.zeros((Hst.m, Hst.n), dtype=torch.float32, device=dev)
rows = torch.repeat_interleave(torch.arange(Hst.m, device=dev),
                               torch.from_numpy(np.diff(Hst.row_ptr).astype(np.int64)).to(dev))
Hd[rows, torch.from_numpy(np.asarray(Hst.col_idx, dtype=np.int64)).to(dev)] = 1.0
e = (torch.rand((B, Hst.n), generator=g, device=dev) < p).to(torch.float32)
synd = (torch.remainder(e @ Hd.t(), 2.0)).to(torch.uint8).contiguous()
corr = torch.empty((B, Hst.n), dtype=torch.uint8, device=dev)
iters = torch.empty(B, dtype=torch.int32, device=dev)
conv = torch.empty(B, dtype=torch.uint8, device=dev)
dec.decode_batch_device(synd, corr, iters, conv)
torch.cuda.synchronize(dev)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(3):
    dec.decode_batch_device(synd, corr, iters, conv)
e1.record()
torch.cuda.synchronize(dev)
geo = dec.geometry()
print(json.dumps({"code": name, "t0": t0, "p": p, "syndromes": B, "shape": [Hst.m, Hst.n],
                  "E3_TAIL": os.environ.get("QLDPC_E3_TAIL", "1"), "env": {k: v for k, v in os.environ.items() if k.startswith("QLDPC_")}, "engine": geo["engine"],
                  "kernel_id": geo["kernel_id"], "threads": geo["threads"], "vpl": geo["vars_per_thread"],
                  "lds_bytes": geo["lds_bytes"], "ms": e0.elapsed_time(e1) / 3,
                  "mean_iters": float(iters.float().mean())}))
