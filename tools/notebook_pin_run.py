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


def cell_counts(cell: int, mult: float, seed: int, precision: int = 64, log=print, hyp: str = "H0_q0"):
    """{rounds: {"samples": S, "fail": [[...codes...][...p...]], "K": [...]}} for one cell under
    one of ``notebook_pin.HYPOTHESES`` (q = q_frac·p syndrome flips, R - 1 + round_shift noisy
    rounds, final-round OSD method / order)."""
    h = nbp.HYPOTHESES[hyp]
    osd_method, osd_order = h["osd"]
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
                                prm["alpha"], osd_method, osd_order, precision=precision)
            d2z = BPOSD_Decoder(code.hx, (probs[1] + probs[2]) * np.ones(code.N), prm["max_iter2"], "minimum_sum",
                                prm["alpha"], osd_method, osd_order, precision=precision)
            sim = CodeSimulator_Phenon(code=code, decoder1_x=d1x, decoder1_z=d1z, decoder2_x=d2x, decoder2_z=d2z,
                                       pauli_error_probs=probs, q=h["q_frac"] * p,
                                       seed=seed + 1000 * cell + 100 * ci + pi)
            assert sim._engine_parts() is not None and all(o is not None for o in sim._final_osd())
            for R in spec["rounds"]:
                res = sim.fused_counts(R + h["round_shift"], out[R]["samples"])
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
                    "A_pct": nbp.percentile_of(A0, fits[:, 0]), "p_c_pct": nbp.percentile_of(pc0, fits[:, 1]),
                    "A_mid": nbp.mid_percentile(A0, fits[:, 0]), "p_c_mid": nbp.mid_percentile(pc0, fits[:, 1])}
            try:
                wer = np.vstack([nbp.WER_FORMULAS[f](fp[i] * c["samples"], c["samples"], c["K"][i], R)
                                 for i in range(len(c["K"]))])
                e[f]["fit_at_engine_rates"] = nbp.threshold_est(P, wer)
            except Exception as ex:  # noqa: BLE001
                e[f]["fit_at_engine_rates"] = repr(ex)
        rep[R] = e
    return rep


def hypothesis_table(cells_bands: dict, formula: str = "current") -> dict:
    """Uniformity of the 15 printed (A, p_c) mid-rank percentiles under one hypothesis."""
    pc = [e[formula]["p_c_mid"] for b in cells_bands.values() for e in b.values()]
    A = [e[formula]["A_mid"] for b in cells_bands.values() for e in b.values()]
    inside = sum(bool(e[formula]["p_c_in"]) for b in cells_bands.values() for e in b.values())
    per_cell = {str(c): nbp.uniformity([e[formula]["p_c_mid"] for e in b.values()]) for c, b in cells_bands.items()}
    return {"p_c": nbp.uniformity(pc), "A": nbp.uniformity(A), "p_c_inside_95": inside, "n": len(pc),
            "p_c_pcts": pc, "A_pcts": A, "per_cell_p_c": per_cell}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, nargs="+", default=[16, 20, 25])
    ap.add_argument("--hyp", nargs="+", default=["H0_q0"],
                    help=f"any of {list(nbp.HYPOTHESES)}, or 'adopted' (notebook_pin.ADOPTED per cell)")
    ap.add_argument("--mult", type=float, default=25.0)
    ap.add_argument("--draws", type=int, default=400)
    ap.add_argument("--seed", type=int, default=0x5EED)
    ap.add_argument("--precision", type=int, default=64)
    ap.add_argument("--out", default="gpurun_out/pin/pin.json")
    ap.add_argument("--counts-only", action="store_true", help="GPU counts only (bands later, on the host)")
    ap.add_argument("--bands-from", default=None, help="recompute bands / tables from a counts file (no GPU)")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    if a.bands_from:
        src = json.load(open(a.bands_from))
        for hyp, hres in src["hypotheses"].items():
            for cell, v in hres["cells"].items():
                cnt = {int(R): c for R, c in v["counts"].items()}
                v["bands"] = bands(int(cell), cnt, a.draws)
            hres["table"] = {fm: hypothesis_table({c: v["bands"] for c, v in hres["cells"].items()}, fm)
                             for fm in ("current", "commented")}
            _report(hyp, hres)
        src["draws"] = a.draws
        with open(a.out, "w") as f:
            json.dump(src, f, indent=1)
        return
    result = {"mult": a.mult, "draws": a.draws, "seed": a.seed, "precision": a.precision, "hypotheses": {}}
    for hyp in a.hyp:
        hres = {"spec": ({str(c): nbp.ADOPTED[c] for c in a.cells} if hyp == "adopted" else nbp.HYPOTHESES[hyp]),
                "cells": {}}
        result["hypotheses"][hyp] = hres
        for cell in a.cells:
            t0 = time.time()
            h_cell = nbp.ADOPTED[cell] if hyp == "adopted" else hyp
            cnt = cell_counts(cell, a.mult, a.seed, a.precision, log=lambda s: print(hyp, s, flush=True), hyp=h_cell)
            hres["cells"][str(cell)] = {"counts": {str(R): v for R, v in cnt.items()},
                                        "gpu_seconds": time.time() - t0}
            if not a.counts_only:
                hres["cells"][str(cell)]["bands"] = bands(cell, cnt, a.draws)
            with open(a.out, "w") as f:
                json.dump(result, f, indent=1)
        if a.counts_only:
            continue
        hres["table"] = {fm: hypothesis_table({c: v["bands"] for c, v in hres["cells"].items()}, fm)
                         for fm in ("current", "commented")}
        with open(a.out, "w") as f:
            json.dump(result, f, indent=1)
        _report(hyp, hres)


def _report(hyp, hres):
    t = hres["table"]["current"]
    print(f"== {hyp}: p_c KS p={t['p_c']['ks_p']:.4g} Fisher p={t['p_c']['fisher_p']:.4g} "
          f"mean pct={t['p_c']['mean']:.3f} inside95={t['p_c_inside_95']}/{t['n']}; "
          f"A KS p={t['A']['ks_p']:.4g} Fisher p={t['A']['fisher_p']:.4g}", flush=True)
    print("   p_c pcts:", " ".join(f"{x:.3f}" for x in t["p_c_pcts"]), flush=True)


if __name__ == "__main__":
    main()
