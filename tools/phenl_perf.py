"""Throughput of the phenomenological space-time shot loop (BASELINE config 5).

hgp_34_n1225_q3 stand-in, num_rep=3, num_cycles=13 (num_rounds=5), p_data = q =
eval_p, Pauli [eval_p/2]*3, min-sum alpha=0.625, max_iter=int(n/10).  Usage:
python tools/phenl_perf.py [code] [eval_p,...] [samples] [precision]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from qldpc_fault_tolerance_amd import codes  # noqa: E402
from qldpc_fault_tolerance_amd.engine import DeviceBP, DevicePhenl, MCResult  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "hgp_34_n1225_q3"
ps = [float(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0.01,0.02,0.03").split(",")]
S = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
prec = int(sys.argv[4]) if len(sys.argv) > 4 else 32
rep, cycles = 3, 13
R = int((cycles - 1) / rep + 1)
code = codes.get_code(name)
n = code.N
mi = int(n / 10)
for p in ps:
    hz, hx = code.csr("hz"), code.csr("hx")
    st_x = DeviceBP(codes.space_time_csr(code.hz, rep), np.hstack([p * np.ones(n), p * np.ones(hz.m)] * rep),
                    max_iter=mi, precision=prec)
    st_z = DeviceBP(codes.space_time_csr(code.hx, rep), np.hstack([p * np.ones(n), p * np.ones(hx.m)] * rep),
                    max_iter=mi, precision=prec)
    d2x = DeviceBP(hz, p * np.ones(n), max_iter=mi, precision=prec)
    d2z = DeviceBP(hx, p * np.ones(n), max_iter=mi, precision=prec)
    ph = DevicePhenl(code, st_x, st_z, d2x, d2z, num_rep=rep, max_batch=S)
    cnt = ph.new_counters()
    ph.launch(p / 2, p / 2, p / 2, p, 1, 0, min(S, 4096), R, "Total", cnt)  # warmup
    torch.cuda.synchronize()
    cnt.zero_()
    t0 = time.perf_counter()
    ph.launch(p / 2, p / 2, p / 2, p, 1, 10**9, S, R, "Total", cnt)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    r = MCResult.from_words(cnt.cpu().numpy())
    dec = sum(r.sector_decodes)
    print(json.dumps({"code": name, "eval_p": p, "samples": S, "num_rounds": R, "num_rep": rep, "precision": prec,
                      "st_engine": st_x.geometry()["engine"], "seconds": dt, "samples_per_s": S / dt,
                      "decodes_per_s": dec / dt, "mean_iters": sum(r.sector_iters) / dec,
                      "nonconv_frac": sum(r.sector_nonconv) / dec, "ler": r.failures / S}), flush=True)
