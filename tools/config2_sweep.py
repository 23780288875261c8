"""BASELINE config 2: the code-capacity threshold sweep over p on one MI355X.

The ``CodeFamily.EvalWER('data')`` point (src/Simulators.py:759-777) for each (code, p):
decoders on hz / hx with ``p_data = eval_p`` (min-sum, alpha 0.625, max_iter int(N/10)),
depolarizing ``[eval_p/2]*3``, ``eval_logical_type='Total'``; shots through the fused engine
(``DeviceMC``) in launches of ``--chunk`` shots with the counters kept on the device.  One
JSON line per point: LER with its 95 % Wilson interval, WER (A8 formula), mean iterations
per decode, non-converged fraction, shots/s.

    python tools/config2_sweep.py --codes hgp_34_n1600 --shots 1e8 --out gpurun_out/c2/n1600.jsonl
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

P_GRID = [float(x) for x in np.geomspace(0.02, 0.12, 10)]  # 10 log-spaced p on [0.02, 0.12]


def wilson(k: int, n: int, z: float = 1.959963984540054):
    if n == 0:
        return (0.0, 1.0)
    ph = k / n
    den = 1 + z * z / n
    c = (ph + z * z / (2 * n)) / den
    h = z * math.sqrt(ph * (1 - ph) / n + z * z / (4 * n * n)) / den
    return (max(0.0, c - h), min(1.0, c + h))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--codes", nargs="+", default=["hgp_34_n1600"])
    ap.add_argument("--shots", type=float, default=1e8)
    ap.add_argument("--p", type=float, nargs="*", default=None)
    ap.add_argument("--precision", type=int, default=64)
    ap.add_argument("--chunk", type=int, default=1 << 22)
    ap.add_argument("--seed", type=int, default=0x51D5EED2)
    ap.add_argument("--out", default="gpurun_out/c2/sweep.jsonl")
    a = ap.parse_args()
    import torch

    from qldpc_fault_tolerance_amd import codes
    from qldpc_fault_tolerance_amd.engine import DeviceBP, DeviceMC, MCResult

    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    P = a.p if a.p else P_GRID
    S = int(a.shots)
    for name in a.codes:
        code = codes.get_code(name)
        n = code.N
        mi = int(n / 10)
        for ep in P:
            dx = DeviceBP(code.hz, ep * np.ones(n), max_iter=mi, precision=a.precision)
            dz = DeviceBP(code.hx, ep * np.ones(n), max_iter=mi, precision=a.precision,
                          vars_per_thread=dx.geometry()["vars_per_thread"])
            mc = DeviceMC(code, dx, dz)
            cnt = mc.new_counters()
            pp = ep / 2
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tp = t0
            for s0 in range(0, S, a.chunk):
                mc.launch(pp, pp, pp, a.seed, s0, min(a.chunk, S - s0), "Total", cnt)
                if time.perf_counter() - tp > 30:  # progress line (keeps a long point visibly alive)
                    torch.cuda.synchronize()
                    tp = time.perf_counter()
                    print(f"  {name} p={ep:.4f}: {s0 + min(a.chunk, S - s0)} / {S} shots, {tp - t0:.0f} s", flush=True)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            r = MCResult.from_words(cnt.cpu().numpy())
            ler = r.failures / r.shots
            lo, hi = wilson(r.failures, r.shots)
            dec = sum(r.sector_decodes)
            line = {"code": name, "N": n, "K": code.K, "eval_p": ep, "precision": a.precision, "shots": r.shots,
                    "failures": r.failures, "ler": ler, "ler_ci95": [lo, hi],
                    "wer": 1.0 - (1 - ler) ** (1 / code.K), "wer_ci95": [1.0 - (1 - lo) ** (1 / code.K),
                                                                        1.0 - (1 - hi) ** (1 / code.K)],
                    "mean_iters": sum(r.sector_iters) / dec, "nonconv_frac": sum(r.sector_nonconv) / dec,
                    "max_iter": mi, "seconds": dt, "shots_per_s": r.shots / dt, "seed": a.seed}
            with open(a.out, "a") as f:
                f.write(json.dumps(line) + "\n")
            print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
