"""Sum rocprofv3 PMC counters of the MC kernel over every pass directory: python tools/pmc_summary.py <dir> [kernel-substr]."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "mc_kernel"
agg = collections.OrderedDict()
disp = collections.defaultdict(set)
for f in sorted(glob.glob(os.path.join(d, "p*", "p_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            disp[r["Counter_Name"]].add(r["Dispatch_Id"])
for k, v in agg.items():
    print(f"{k:26s} {v:.6g}  (dispatches: {len(disp[k])})")
