"""Dump the lane map of the headline m2s decoders for tools/dev/place_opt.cpp (host only, no GPU).

Restates the engine's engine-3 slot map for the m2s family (qldpc_hip.hip: variables sorted by
column degree, degree <= 3 first, natural order inside a class; slot k of lane t holds variable
slot_var[k * TB + t]) and writes: m n TB VPL DM D3K, slot_var, then per variable its rows ascending.

    python tools/dev/place_dump.py hz > /tmp/hz.txt
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from qldpc_fault_tolerance_amd import codes  # noqa: E402

sec = sys.argv[1] if len(sys.argv) > 1 else "hz"
name = sys.argv[2] if len(sys.argv) > 2 else "hgp_34_n1600"
H = getattr(codes.get_code(name), sec)
m, n = H.shape
TB, VPL, DM = 256, 7, 4
deg = H.sum(0).astype(int)
order = [j for j in range(n) if deg[j] <= 3] + [j for j in range(n) if deg[j] > 3]
sv = order + [-1] * (VPL * TB - n)
d3k = 0
for k in range(VPL):
    if all(j < 0 or deg[j] <= 3 for j in sv[k * TB:(k + 1) * TB]):
        d3k = k + 1
    else:
        break
out = [f"{m} {n} {TB} {VPL} {DM} {d3k}", " ".join(map(str, sv))]
for j in range(n):
    rows = np.flatnonzero(H[:, j])
    out.append(f"{len(rows)} " + " ".join(map(str, rows)))
print("\n".join(out))
