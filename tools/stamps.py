"""Phase shares of the fused MC kernel (or, --st, config 5's space-time decode_batch) from a
QLDPC_STAMPS diagnostic build.

    python tools/build_variant.py libqldpc_hip_stamps.so QLDPC_STAMPS=1
    QLDPC_LIB=$PWD/qldpc_fault_tolerance_amd/libqldpc_hip_stamps.so python tools/stamps.py [prof_one args]

Runs one launch like tools/prof_one.py and prints the per-wave cycle shares of the variable
phase, its barrier, the check phase, the flags barrier, shot setup and epilogue.  Read the
shares, not the absolute time (the stamps' waits forbid overlaps of the real kernel).
"""
import ctypes
import os
import runpy
import sys

here = os.path.dirname(os.path.abspath(__file__))
# --st: one space-time decode_batch launch of config 5 (tools/prof_st.py args) instead of the fused MC
st = len(sys.argv) > 1 and sys.argv[1] == "--st"
sys.argv = [os.path.join(here, "prof_st.py" if st else "prof_one.py")] + sys.argv[(2 if st else 1):]
runpy.run_path(sys.argv[0], run_name="__main__")
from qldpc_fault_tolerance_amd import _native  # noqa: E402

lib = ctypes.CDLL(_native.LIB_PATH)
out = (ctypes.c_ulonglong * 10)()
assert lib.qldpc_debug_stamps(out) == 0
v = list(out)
names = ["var", "var_barrier", "check", "flag_barrier", "setup_sample", "epilogue", "", "", "setup_prev_bar",
         "first_check"]
tot = sum(v[:6]) + v[8] + v[9]
its, shots = v[6], v[7]
print(f"wave-iterations {its}  wave-shots {shots}  iters/shot {its / max(1, shots):.1f}")
for k, nm in enumerate(names):
    if not nm:
        continue
    per = v[k] / max(1, its if k < 4 else shots)
    print(f"{nm:14s} {100 * v[k] / tot:6.2f}%  {per:9.1f} clk per {'iteration' if k < 4 else 'shot'}")
