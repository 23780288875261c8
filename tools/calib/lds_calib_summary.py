"""Summarize tools/calib/lds_calib's JSON lines into profiles/r04/calib/lds_calib.json (bench.py's
measured LDS mix peak for the headline m2s family).

    python tools/calib/lds_calib_summary.py gpurun_out/<dir>/calib.jsonl [more.jsonl ...]

peak = the highest rate any row-mix mode reached (mix / mix_pipe / mix_pipe2 / mix_pipe4), in
ALGORITHMIC bytes (224 B per row of 7 edges; the mix moves 240 B of LDS transfer per row), over
all given runs.  The guide's 75 TB/s aggregate stays bench.py's `peak_guide`.
"""
import json
import os
import sys

runs = []
for path in sys.argv[1:]:
    lines = [json.loads(x) for x in open(path) if x.strip().startswith("{")]
    runs.append({"file": path, "modes": {d["mode"]: d for d in lines if "mode" in d}, "setup": lines[0]})
best, where = 0.0, None
for r in runs:
    for name, d in r["modes"].items():
        if name.startswith("mix") and d.get("algorithmic_TBps", 0) > best:
            best, where = d["algorithmic_TBps"], (r["file"], name)
out = {"mix_peak_algorithmic_GBs": best * 1000.0, "mix_peak_transfer_GBs": best * 1000.0 * 240 / 224,
       "mode": where[1], "source": where[0],
       "what": "tools/calib/lds_calib.hip: the m2s kernel's per-row LDS mix (15 ds_read_b64 + 3 ds_read_b128 + "
               "9 ds_write_b64 per lane-row), 3 x 256-thread workgroups with 52 KiB images per CU, conflict-free "
               "addresses, loads and stores software-pipelined; algorithmic bytes = 224 per row",
       "runs": [{"file": r["file"], "modes": {k: {kk: v[kk] for kk in ("TBps", "algorithmic_TBps", "ms") if kk in v}
                                                 for k, v in r["modes"].items()}} for r in runs],
       "counter_calibration": "SQ_INSTS_LDS_LOAD_BANDWIDTH / STORE_BANDWIDTH x 64 B = the exact bytes moved by "
                              "lds_mix<0> (2004 iterations: 6.619e10 B read, ratio 1.000; store within the "
                              "image-init bytes), profiles/r04/calib/lds_calib_pmc.csv"}
os.makedirs("profiles/r04/calib", exist_ok=True)
json.dump(out, open("profiles/r04/calib/lds_calib.json", "w"), indent=1)
print(json.dumps({k: out[k] for k in ("mix_peak_algorithmic_GBs", "mode", "source")}))
