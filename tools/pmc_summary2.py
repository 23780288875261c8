"""Summarise rocprofv3 --pmc pass CSVs (tools/pmc_passes.sh output) for the dominant kernel:
python tools/pmc_summary2.py <outdir>  -> counter totals + derived ratios."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
tot = defaultdict(float)
kern = None
for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "")
        if "rmc_kernel" not in k and "rdec_kernel" not in k and "hmc_kernel" not in k and "hdec_kernel" not in k:
            continue
        kern = k
        tot[row["Counter_Name"]] += float(row["Counter_Value"])
print(kern)
for k in sorted(tot):
    print(f"{k:28s} {tot[k]:.4g}")
g = tot.get
if g("SQ_WAVE_CYCLES"):
    wc = g("SQ_WAVE_CYCLES")
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
        if g(k):
            print(f"{k}/WAVE_CYCLES = {g(k) / wc:.3f}")
if g("SQ_LDS_IDX_ACTIVE"):
    print(f"LDS_BANK_CONFLICT/LDS_IDX_ACTIVE = {g('SQ_LDS_BANK_CONFLICT', 0) / g('SQ_LDS_IDX_ACTIVE'):.3f}")
if g("SQ_INSTS_LDS") and g("SQ_INSTS_VALU"):
    print(f"VALU:LDS = {g('SQ_INSTS_VALU') / g('SQ_INSTS_LDS'):.2f}")
