"""One space-time decode_batch launch of BASELINE config 5's decoder (for rocprofv3 --pmc passes).

    python tools/prof_st.py [p] [syndromes] [precision] [code] [seed]

Builds the hz space-time decoder exactly as bench.py --workload phenl does (hgp_34_n1225_q3,
num_rep 3, min-sum alpha 0.625, max_iter int(n/10)) and decodes ``syndromes`` syndromes of i.i.d.
errors at rate p on the stacked graph, as bench.py's st_kernel_roofline does (one warm-up launch,
then one launch).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from qldpc_fault_tolerance_amd import codes  # noqa: E402
from qldpc_fault_tolerance_amd.engine import DeviceBP  # noqa: E402

p = float(sys.argv[1]) if len(sys.argv) > 1 else 0.06
B = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
prec = int(sys.argv[3]) if len(sys.argv) > 3 else 32
name = sys.argv[4] if len(sys.argv) > 4 else "hgp_34_n1225_q3"
seed = int(sys.argv[5]) if len(sys.argv) > 5 else 20240611 + 11
rep = 3
code = codes.get_code(name)
n = code.N
hz = code.csr("hz")
Hst = codes.space_time_csr(code.hz, rep)
dec = DeviceBP(Hst, np.hstack([p * np.ones(n), p * np.ones(hz.m)] * rep), max_iter=int(n / 10), precision=prec)
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(seed)
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
dec.decode_batch_device(synd, corr, iters, conv)
torch.cuda.synchronize(dev)
print("geometry", dec.geometry(), "mean iters", float(iters.float().mean()))
