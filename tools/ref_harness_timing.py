"""Cost of the reference's own Python harness on this host.

BUILD CONTAINER ONLY (reads /root/reference; never shipped to or run on the GPU box).  Imports the
reference's ``Simulators`` / ``Decoders`` with the stub modules of ``tests/golden/make_golden.py``
and times ``CodeSimulator_DataError._single_run`` on the bench workload (hgp_34_n1600 stand-in,
eval_p = 0.06, ``BP_Decoder_Class(10, "minimum_sum", 0.625)`` decoders = the reference factory)
with the repository's C oracle standing in for the absent ``ldpc.bp_decoder`` — so the number is
the reference harness (Python error loop, dense float64 matvecs, failure checks) around a native
BP of ldpc's arithmetic, one process, one core.  Also times the harness alone (a zero decoder).

    python tools/ref_harness_timing.py [shots] > profiles/r04/ref_harness_timing.json
"""
from __future__ import annotations

import json
import os
import platform
import random
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

import numpy as np  # noqa: E402

import make_golden as mg  # noqa: E402  (stub installer + OracleBP)


def cpu_model():
    for line in open("/proc/cpuinfo"):
        if line.lower().startswith("model name"):
            return line.split(":", 1)[1].strip()
    return platform.processor()


def main():
    shots = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    mg.install_stubs()
    import Decoders
    import Simulators

    code = mg.codes.get_code("hgp_34_n1600")
    p = 0.06
    pp = p * 3 / 2 / 3
    cls = Decoders.BP_Decoder_Class(max_iter_ratio=10, bp_method="minimum_sum", ms_scaling_factor=0.625)
    dx = cls.GetDecoder({"h": code.hz, "p_data": p})
    dz = cls.GetDecoder({"h": code.hx, "p_data": p})
    sim = Simulators.CodeSimulator_DataError(code=code, decoder_x=dx, decoder_z=dz, pauli_error_probs=[pp] * 3,
                                             eval_logical_type="Total")
    random.seed(12345)
    sim._single_run()  # warm-up (CSR conversion of the stubbed decoders)
    t0 = time.perf_counter()
    fails = sum(sim._single_run() for _ in range(shots))
    dt = time.perf_counter() - t0

    class Zero:
        def decode(self, synd):
            return np.zeros(code.N, dtype=int)

    sim0 = Simulators.CodeSimulator_DataError(code=code, decoder_x=Zero(), decoder_z=Zero(), pauli_error_probs=[pp] * 3,
                                              eval_logical_type="Total")
    n0 = max(50, shots)
    t1 = time.perf_counter()
    for _ in range(n0):
        sim0._single_run()
    dt0 = time.perf_counter() - t1
    print(json.dumps({
        "what": "reference _single_run (src/Simulators.py:117-168) stub-imported, oracle C BP standing in for ldpc",
        "workload": "hgp_34_n1600 stand-in, eval_p=0.06, BP_Decoder_Class(10, minimum_sum, 0.625), Total",
        "shots": shots, "seconds": dt, "shots_per_s_one_core": shots / dt, "ms_per_shot": dt / shots * 1e3,
        "ler": fails / shots,
        "harness_only_ms_per_shot": dt0 / n0 * 1e3, "harness_only_note": "zero decoder: error loop + 4 dense matvecs",
        "cpu_model": cpu_model(), "cores_used": 1, "host": "build container (8 CPUs, no GPU)"}, indent=1))


if __name__ == "__main__":
    main()
