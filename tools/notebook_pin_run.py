"""GPU side of the notebook pin (tests/notebook_pin.py): failure counts of the
Threshold notebook's phenomenological cells on the engine, then the bootstrap
bands of the notebook's printed (A, p_c).

    python tools/notebook_pin_run.py --cells 16 20 25 --mult 25 --out gpurun_out/pin/pin.json

Each (code, p) point is ``CodeFamilyPhenlThreshold`` (Threshold-checkpoint.ipynb
lines 127-170) on the drop-in classes: CodeSimulator_Phenon (q = 0), BPDecoder on
[h | I] (int(N/30)), BPOSD_Decoder OSD-E(10) (int(N/10)); ``mult`` × the notebook's
sample count per round count.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import notebook_pin as nbp  # noqa: E402


def cell_counts(cell: int, mult: float, seed: int, precision: int = 64, log=print):
    """{rounds: {"samples": S, "fail": [[...codes...][...p...]], "K": [...]}} for one cell."""
    from qldpc_fault_tolerance_amd.decoders import BPDecoder, BPOSD_Decoder
    from qldpc_fault_tolerance_amd.simulators import CodeSimulator_Phenon

    spec = nbp.CELLS[cell]
    P = nbp.cell_p_list(cell)
    out = {R: {"samples": int(round(mult * nbp.cell_samples(cell, R))), "fail": [], "K": []} for R in spec["rounds"]}
    for ci, name in enumerate(spec["codes"]):
        code = nbp.cell_code(name)
        prm = nbp.decoder_params(code.N)
        hx_ext = np.hstack([code.hx, np.identity(code.hx.shape[0])])
        hz_ext = np.hstack([code.hz, np.identity(code.hz.shape[0])])
        rows = {R: [] for R in spec["rounds"]}
        for pi, p in enumerate(P):
            probs = [p / 3, p / 3, p / 3]
            t0 = time.time()
            d1x = BPDecoder(hz_ext, (probs[0] + probs[1]) * np.ones(hz_ext.shape[1]), prm["max_iter1"],
                            "minimum_sum", prm["alpha"], precision=precision)
            d1z = BPDecoder(hx_ext, (probs[0] + probs[1]) * np.ones(hx_ext.shape[1]), prm["max_iter1"],
                            "minimum_sum", prm["alpha"], precision=precision)
            d2x = BPOSD_Decoder(code.hz, (probs[0] + probs[1]) * np.ones(code.N), prm["max_iter2"], "minimum_sum",
                                prm["alpha"], "osd_e", prm["osd_order"], precision=precision)
            d2z = BPOSD_Decoder(code.hx, (probs[1] + probs[2]) * np.ones(code.N), prm["max_iter2"], "minimum_sum",
                                prm["alpha"], "osd_e", prm["osd_order"], precision=precision)
            sim = CodeSimulator_Phenon(code=code, decoder1_x=d1x, decoder1_z=d1z, decoder2_x=d2x, decoder2_z=d2z,
                                       pauli_error_probs=probs, seed=seed + 1000 * cell + 100 * ci + pi)
            assert sim._engine_parts() is not None and all(o is not None for o in sim._final_osd())
            for R in spec["rounds"]:
                res = sim.fused_counts(R, out[R]["samples"])
                rows[R].append(int(res.failures))
            log(f"cell {cell} {name} p={p:.4f}: " + " ".join(f"R{R}:{rows[R][-1]}/{out[R]['samples']}"
                                                            for R in spec["rounds"]) + f"  ({time.time() - t0:.1f}s)")
        for R in spec["rounds"]:
            out[R]["fail"].append(rows[R])
            out[R]["K"].append(int(code.K))
    return out


def bands(cell: int, counts: dict, draws: int, formulas=("commented", "current")):
    P = nbp.cell_p_list(cell)
    rep = {}
    for R, c in counts.items():
        R = int(R)
        fp = np.asarray(c["fail"], dtype=np.float64) / c["samples"]
        A0, pc0, line = nbp.PRINTED[cell][R]
        e = {"printed": {"A": A0, "p_c": pc0, "line": line}, "fail_prob": fp.tolist(), "samples": c["samples"],
             "notebook_samples": nbp.cell_samples(cell, R)}
        for f in formulas:
            b = nbp.bootstrap_band(fp, c["K"], P, nbp.cell_samples(cell, R), R, formula=f, draws=draws,
                                   seed=17 + R + cell)
            fits = b["fits"]
            e[f] = {"A_band": b.get("A"), "p_c_band": b.get("p_c"), "failed_fits": b["failed"], "draws": b["draws"],
                    "A_in": nbp.inside(A0, b.get("A")), "p_c_in": nbp.inside(pc0, b.get("p_c")),
                    "A_pct": nbp.percentile_of(A0, fits[:, 0]), "p_c_pct": nbp.percentile_of(pc0, fits[:, 1])}
            try:
                wer = np.vstack([nbp.WER_FORMULAS[f](fp[i] * c["samples"], c["samples"], c["K"][i], R)
                                 for i in range(len(c["K"]))])
                e[f]["fit_at_engine_rates"] = nbp.threshold_est(P, wer)
            except Exception as ex:  # noqa: BLE001
                e[f]["fit_at_engine_rates"] = repr(ex)
        rep[R] = e
    return rep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, nargs="+", default=[16, 20, 25])
    ap.add_argument("--mult", type=float, default=25.0)
    ap.add_argument("--draws", type=int, default=400)
    ap.add_argument("--seed", type=int, default=0x5EED)
    ap.add_argument("--precision", type=int, default=64)
    ap.add_argument("--out", default="gpurun_out/pin/pin.json")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    result = {"mult": a.mult, "draws": a.draws, "seed": a.seed, "precision": a.precision, "cells": {}}
    for cell in a.cells:
        t0 = time.time()
        cnt = cell_counts(cell, a.mult, a.seed, a.precision, log=lambda s: print(s, flush=True))
        result["cells"][cell] = {"counts": {str(R): v for R, v in cnt.items()}, "gpu_seconds": time.time() - t0,
                                 "bands": bands(cell, cnt, a.draws)}
        with open(a.out, "w") as f:
            json.dump(result, f, indent=1)
        for R, e in result["cells"][cell]["bands"].items():
            pr = e["printed"]
            msg = [f"cell {cell} R={R} printed A={pr['A']:.4g} p_c={pr['p_c']:.4g} (line {pr['line']})"]
            for fm in ("commented", "current"):
                x = e[fm]
                msg.append(f"  [{fm}] A band {x['A_band']} in={x['A_in']} pct={x['A_pct']:.3f}; p_c band "
                           f"{x['p_c_band']} in={x['p_c_in']} pct={x['p_c_pct']:.3f}; failed {x['failed_fits']}")
            print("\n".join(msg), flush=True)


if __name__ == "__main__":
    main()
