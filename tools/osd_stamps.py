"""Step shares of osd_gpu_kernel from a QLDPC_STAMPS diagnostic build:

    python tools/build_variant.py libqldpc_hip_stamps.so QLDPC_STAMPS=1
    QLDPC_LIB=$PWD/qldpc_fault_tolerance_amd/libqldpc_hip_stamps.so python tools/osd_stamps.py [code] [p] [shots] [precision]

Runs the device-resident BP+OSD-E(10) shot loop (bench.py --workload bposd) once and prints the
per-workgroup cycle shares of the OSD kernel's steps.  Shares only (the stamps' waits forbid
overlaps the real kernel has).
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from qldpc_fault_tolerance_amd import _native, codes  # noqa: E402
from qldpc_fault_tolerance_amd.decoders import BPOSD_Decoder_Class  # noqa: E402
from qldpc_fault_tolerance_amd.simulators import CodeSimulator_DataError  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "hgp_34_n1600"
p = float(sys.argv[2]) if len(sys.argv) > 2 else 0.04
S = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
prec = int(sys.argv[4]) if len(sys.argv) > 4 else 64
code = codes.get_code(name)
cls = BPOSD_Decoder_Class(10, "minimum_sum", 0.625, "osd_e", 10, precision=prec)
dx, dz = cls.GetDecoder({"h": code.hz, "p_data": p}), cls.GetDecoder({"h": code.hx, "p_data": p})
sim = CodeSimulator_DataError(code, dx, dz, [p / 2] * 3, "Total", seed=5)
lib = ctypes.CDLL(_native.LIB_PATH)
out = (ctypes.c_ulonglong * 16)()
sim.bposd_counts(S)  # warm-up
assert lib.qldpc_debug_osd_stamps(out) == 0
f, c, o = sim.bposd_counts(S)
assert lib.qldpc_debug_osd_stamps(out) == 0
v = list(out)
names = ["sort", "H load", "Gauss-Jordan", "swaps + bit-vectors", "candidates", "outputs"]
tot = sum(v[:6])
print(f"{name} p={p} shots={c} osd decodes={o} syndromes stamped={v[6]}")
for k, nm in enumerate(names):
    print(f"{nm:20s} {100 * v[k] / max(1, tot):6.2f}%  {v[k] / max(1, v[6]):10.0f} clk per syndrome")
if os.environ.get("QLDPC_OSD_PNL", "0") in ("1", "2"):  # panel modes: [7] pivots, [8] panel searches, [9] panel updates
    print(f"pivots per syndrome {v[7] / max(1, v[6]):.0f}; per pivot: {v[2] / max(1, v[7]):.0f} clk, "
          f"of which the panel's pivot search {v[8] / max(1, v[7]):.0f}, the panel's row updates {v[9] / max(1, v[7]):.0f}")
else:
    print(f"positions per syndrome {v[7] / max(1, v[6]):.0f}; per position: {v[2] / max(1, v[7]):.0f} clk, "
          f"of which search + barrier {v[8] / max(1, v[7]):.0f}, pivot-row publication + barrier (register rows) "
          f"{v[9] / max(1, v[7]):.0f}")
if os.environ.get("QLDPC_OSD_PNL", "0") == "3":  # blocked: [7] pivots, [8] searches, [9] tables, [10] row updates, [11] step 1
    pv = max(1, v[7])
    print(f"blocked: pivots per syndrome {v[7] / max(1, v[6]):.0f}; per pivot: search {v[8] / pv:.0f} clk, tables {v[9] / pv:.0f}, "
          f"row updates {v[10] / pv:.0f}, panel-word exchange {v[11] / pv:.0f} (Gauss-Jordan {v[2] / pv:.0f})")
if os.environ.get("QLDPC_OSD_PNL", "0") == "5":  # forward: [15] compactions, [13] back substitution (wave 0's view)
    print(f"forward: compactions {v[15] / max(1, v[6]):.0f} clk per syndrome, "
          f"back substitution {v[13] / max(1, v[6]):.0f} clk per syndrome")
