"""MI355X-native Monte Carlo BP decoding engine for quantum LDPC codes.

Drop-in for the hot path of deltaXdeltaQ/QLDPC_Fault_Tolerance
(``src/Simulators.py`` / ``src/Decoders.py`` / ``src/Decoders_SpaceTime.py``):
sample errors, compute syndromes, BP-decode, check logical failures — in
hand-written HIP kernels for gfx950 behind a C ABI (``include/qldpc_hip.h``).
"""
from . import codes, gf2  # noqa: F401

__version__ = "0.1.0"
