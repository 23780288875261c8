"""Fold rocprofv3 FETCH_SIZE / WRITE_SIZE passes of bench.py into profiles/traffic.json.

    python tools/traffic_update.py <run_dir> [code p shots logical precision]

<run_dir> holds pmc_FETCH_SIZE/ and pmc_WRITE_SIZE/ (tools/gpu_round.sh).  Per
MI355X_MICROARCH.md §HBM: FETCH_SIZE x2 on gfx950, WRITE_SIZE as is (KB = 1024 B);
the value is per launch of the headline kernel (rmc_kernel / smc_kernel).
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
run = sys.argv[1]
key = "|".join(sys.argv[2:7]) if len(sys.argv) >= 7 else "hgp_34_n1600|0.06|262144|Total|32"


def per_launch(counter):
    vals, kern = [], None
    for f in glob.glob(os.path.join(run, f"pmc_{counter}", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "mc_kernel" in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
                kern = r["Kernel_Name"]
    if not vals:
        raise SystemExit(f"no {counter} rows for the MC kernel under {run}")
    return sum(vals) / len(vals), kern


fetch, kern = per_launch("FETCH_SIZE")
write, _ = per_launch("WRITE_SIZE")
path = os.path.join(ROOT, "profiles", "traffic.json")
t = json.load(open(path)) if os.path.exists(path) else {}
t["_doc"] = ("HBM bytes per launch of the headline bench kernel, from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes "
             "(separate runs) of `bench.py --steps 1 --warmup 0`; gfx950 correction per MI355X_MICROARCH.md §HBM: "
             "FETCH_SIZE x2, WRITE_SIZE as is; KB = 1024 B.  Folded by tools/traffic_update.py from " + run)
t[key] = {"fetch_kb": fetch * 2, "write_kb": write, "bytes": int((fetch * 2 + write) * 1024), "kernel": kern}
json.dump(t, open(path, "w"), indent=1)
print(key, t[key])
