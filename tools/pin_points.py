"""Per-point pin of the notebook's threshold data against the engine (CPU only).

The notebook's fit plots carry its per-(code, p) word error rates (digitized by
tools/notebook_digitize.py into tests/golden/notebook_plot_points.json: the real ldpc / bposd run at the
notebook's sample sizes).  Each WER is inverted to the per-sample logical failure rate through the WER
transform (src/Simulators.py:353-360 "current", or the commented :341-351 version) and compared with the
engine's failure rate at 25x the samples (profiles/r04/pin/counts.json: the six simulator-setup
hypotheses of round 4; profiles/r05/pin/heldout_counts.json: the adopted ones at the held-out seed):
z = (LER_notebook - LER_engine) / sd, sd from both binomials and 0.4 px of digitization.  Plots whose
y scale the ticks do not pin (cell 25 R = 6) are left out.

    python tools/pin_points.py [out.json]
"""
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import notebook_pin as nbp  # noqa: E402


def inv_current(w, K, R):
    lo = min(max(w, 0.0), 0.5)
    q = (1 - (1 - 2 * lo) ** R) / 2
    return 1 - (1 - q) ** K


def inv_commented(w, K, R):
    pc = min(max(1 - (1 - w) ** K, 0.0), 0.5)
    return (1 - (1 - 2 * pc) ** R) / 2


INV = {"current": inv_current, "commented": inv_commented}


def zscores(points, cells, inv, which):
    out = []
    for pl in points["plots"]:
        cell, R = pl["cell"], pl["rounds"]
        if cell not in which or pl["y_axis"]["tick_pattern"] != "log-subticks" or str(cell) not in cells:
            continue
        c = cells[str(cell)]["counts"].get(str(R))
        if c is None:
            continue
        K, S, ns = c["K"], c["samples"], nbp.cell_samples(cell, R)
        rel = math.log(10) * 0.4 / abs(pl["y_axis"]["b_px_per_decade"])
        for i in range(3):
            for j, p in enumerate(pl["p"]):
                ler = inv(pl["wer"][i][j], K[i], R)
                le = c["fail"][i][j] / S
                sd = math.sqrt(max(le * (1 - le), 1e-12) * (1 / ns + 1 / S) + (rel * le) ** 2)
                out.append({"cell": cell, "rounds": R, "code": i, "p": p, "ler_notebook": ler, "ler_engine": le,
                            "ratio": ler / le if le > 0 else None, "z": (ler - le) / sd, "occluded": pl["occluded"][i][j]})
    return out


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r06", "pin", "points_vs_hypotheses.json")
    points = json.load(open(os.path.join(ROOT, "tests", "golden", "notebook_plot_points.json")))
    runs = {"r04 selection seed 0x5eed": json.load(open(os.path.join(ROOT, "profiles", "r04", "pin", "counts.json")))["hypotheses"],
            "r05 held-out seed 0x55eed": json.load(open(os.path.join(ROOT, "profiles", "r05", "pin", "heldout_counts.json")))["hypotheses"]}
    res = []
    for run, hyps in runs.items():
        for hyp, hd in hyps.items():
            for tname, inv in INV.items():
                for which, group in (((16, 20), "LP cells 16 + 20"), ((25,), "toric cell 25")):
                    z = zscores(points, hd["cells"], inv, which)
                    if not z:
                        continue
                    zz = np.array([x["z"] for x in z])
                    rat = np.array([x["ratio"] for x in z if x["ratio"]])
                    res.append({"run": run, "hypothesis": hyp, "spec": hd.get("spec"), "wer_transform": tname, "group": group,
                                "points": len(z), "mean_z": float(zz.mean()), "chi2_per_point": float(np.mean(zz ** 2)),
                                "median_ratio_notebook_over_engine": float(np.median(rat)),
                                "ratio_q10_q90": [float(np.quantile(rat, 0.1)), float(np.quantile(rat, 0.9))]})
                    r = res[-1]
                    print(f"{run:26s} {hyp:14s} {tname:9s} {group:16s} n={r['points']:3d} mean z {r['mean_z']:+7.2f} "
                          f"chi2/pt {r['chi2_per_point']:8.2f} median LER ratio {r['median_ratio_notebook_over_engine']:.2f}")
    os.makedirs(os.path.dirname(out_path), exist_ok=True)
    json.dump({"what": __doc__.strip().splitlines()[0], "results": res}, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
