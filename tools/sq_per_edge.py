"""SQ counters of one fused MC launch per edge-iteration (test/diagnostic tool).

    python tools/sq_per_edge.py <pmc-dir> <prof_one.log> [kernel-substr] [code]

Sums every pass's counters for the kernel (tools/pmc_summary.py's rule), reads the decodes and mean
iterations per decode that tools/prof_one.py printed, and divides the wave-level instruction counts
by the launch's edge-iterations / 64 (one wave instruction = 64 lanes): SQ_INSTS_VALU per
edge-iteration is the measured counterpart of tools/valu_breakdown.py's static count.
"""
import collections
import csv
import glob
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

d, log = sys.argv[1], sys.argv[2]
sub = sys.argv[3] if len(sys.argv) > 3 else "rmc_kernel"
name = sys.argv[4] if len(sys.argv) > 4 else "hgp_34_n1600"
agg = collections.OrderedDict()
for f in sorted(glob.glob(os.path.join(d, "p*", "p_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
txt = open(log).read()
m = re.search(r"decodes=(\d+).*iters/decode=([\d.]+)", txt)
dec, it = int(m.group(1)), float(m.group(2))
from qldpc_fault_tolerance_amd import codes  # noqa: E402

code = codes.get_code(name)
nnz = (int(code.hz.sum()) + int(code.hx.sum())) / 2  # mean edges per sector decode
ei = dec * it * nnz
print(f"{name}: {dec} decodes x {it:.2f} iterations x {nnz:.0f} edges = {ei:.4g} edge-iterations")
for k, v in agg.items():
    print(f"{k:28s} {v:.5g}   per edge-iteration x 64: {v * 64 / ei:.3f}")
if "SQ_WAVE_CYCLES" in agg and "SQ_ACTIVE_INST_VALU" in agg:
    print(f"VALU busy share of wave cycles: {agg['SQ_ACTIVE_INST_VALU'] / agg['SQ_WAVE_CYCLES']:.3f}")
