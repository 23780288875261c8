"""Summarise the SQ counter passes of tools/archive/r04_gpu_t.sh for the GPU OSD kernel:
python tools/pmc_osd_summary.py <outdir>  -> counter totals over every osd_gpu_kernel dispatch
and the per-wave / per-cycle ratios DESIGN.md quotes."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
tot = defaultdict(float)
kern = set()
for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "")
        if "osd_gpu_kernel" not in k:
            continue
        kern.add(k)
        tot[row["Counter_Name"]] += float(row["Counter_Value"])
print("\n".join(sorted(kern)))
for k in sorted(tot):
    print(f"{k:24s} {tot[k]:.6g}")
g = tot.get
waves = g("SQ_WAVES", 0)
if waves:
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH"):
        if g(k):
            print(f"{k} per wave = {g(k) / waves:.1f}")
wc = g("SQ_WAVE_CYCLES", 0)
if wc:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
              "SQ_ACTIVE_INST_LDS", "SQ_INST_CYCLES_SALU", "SQ_ACTIVE_INST_MISC", "SQ_WAIT_INST_LDS"):
        if g(k):
            print(f"{k} / SQ_WAVE_CYCLES = {g(k) / wc:.3f}")
if g("SQ_BUSY_CYCLES") and g("GRBM_GUI_ACTIVE"):
    print(f"SQ_BUSY_CYCLES / GRBM_GUI_ACTIVE = {g('SQ_BUSY_CYCLES') / g('GRBM_GUI_ACTIVE'):.3f}")
