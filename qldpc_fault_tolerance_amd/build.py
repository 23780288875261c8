"""In-tree build of the HIP engine (``libqldpc_hip.so``) for gfx950.

``hipcc`` cross-compiles without a GPU.  The two translation units are built in
parallel and linked into one shared library next to this file, so the
``.so`` travels with the repository snapshot to the GPU box.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
REPO = os.path.dirname(PKG_DIR)
OUT = os.path.join(PKG_DIR, "libqldpc_hip.so")
ARCH = os.environ.get("QLDPC_OFFLOAD_ARCH", "gfx950")

HIPCC_FLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
    # exact operation order is part of the contract (bit parity with the oracle):
    # no FMA contraction of the v2c sums / c2v products.
    "-ffp-contract=off",
    # scalar f32 arithmetic: SLP-packed v_pk_add/mul plus their pairing moves
    # cost more issue slots than they save in the BP loops (measured).
    "-fno-slp-vectorize",
    "-I", os.path.join(REPO, "include"),
]


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build the engine)")


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def build_native(force: bool = False, verbose: bool = True, out: str | None = None,
                 defines: tuple = ()) -> str:
    """Build the engine; ``out``/``defines`` build a side variant for A/B timing
    (tools/build_variant.py; loaded through ``QLDPC_LIB``)."""
    OUT = out or globals()["OUT"]
    srcs = sources()
    deps = srcs + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    deps.append(os.path.join(REPO, "include", "qldpc_hip.h"))
    if not force and os.path.exists(OUT) and all(os.path.getmtime(OUT) >= os.path.getmtime(d) for d in deps):
        return OUT
    hipcc = _hipcc()
    objdir = os.path.join(PKG_DIR, "build" if out is None else "build_" + os.path.basename(OUT).replace(".so", ""))
    os.makedirs(objdir, exist_ok=True)
    procs = []
    objs = []
    for s in srcs:
        o = os.path.join(objdir, os.path.basename(s).replace(".hip", ".o"))
        objs.append(o)
        cmd = [hipcc, *HIPCC_FLAGS, *("-D" + d for d in defines), "-c", s, "-o", o]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append(subprocess.Popen(cmd))
    bad = [p.wait() for p in procs]
    if any(bad):
        raise RuntimeError("hipcc compile failed")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT + ".tmp", *objs]
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build_native(force="--force" in sys.argv)
