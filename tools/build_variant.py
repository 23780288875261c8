"""Build a side variant of the engine with extra -D defines for A/B timing.

    python tools/build_variant.py libqldpc_hip_x.so QLDPC_TID_LAUNDER=0
    QLDPC_LIB=$PWD/qldpc_fault_tolerance_amd/libqldpc_hip_x.so python bench.py ...
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from qldpc_fault_tolerance_amd import build  # noqa: E402

out = os.path.join(build.PKG_DIR, sys.argv[1])
print(build.build_native(force=True, verbose=False, out=out, defines=tuple(sys.argv[2:])))
