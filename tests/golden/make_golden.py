"""Generate golden vectors from the reference's own Python harness.

Run in the build container only (``/root/reference`` is not on the GPU box):

    python tests/golden/make_golden.py          # reference_harness_n225.npz
    python tests/golden/make_golden.py phen     # reference_harness_phen_n225.npz
    python tests/golden/make_golden.py configs  # reference_harness_configs.npz (configs 2-5)
    python tests/golden/make_golden.py fits     # reference_fits.npz (threshold tooling)
    python tests/golden/make_golden.py schedules  # reference_circuit_schedules.npz (CX schedules)
    python tests/golden/make_golden.py circuit    # reference_circuit.npz (circuit op lists + fault hypergraphs)

The reference modules import third-party packages that are absent here
(``graph_tools``, ``ldpc``, ``bposd``, ``stim``, …), so empty stub
modules are registered under those names before importing
``Decoders``/``Simulators``/``Decoders_SpaceTime``/``Simulators_SpaceTime`` from
``/root/reference/src``.  The reference's own code then runs unchanged for
everything that does not live in those packages: error sampling
(``_generate_error``), syndromes, failure checks (``_single_run``), the WER
formulas (``WordErrorRate``), ``GetSpaceTimeCheckMat`` and the space-time
detector histories.  The one stubbed class that is exercised, ``ldpc.bp_decoder``,
is backed by this repository's CPU oracle — so BP outputs in these fixtures are
oracle outputs (the reference pins no BP results), while
everything around BP is the reference's own behaviour.

No pickle from the reference is loaded: the n225 code comes from the bundled
``.npz`` (converted by the non-executing reader in ``safepickle.py``).
Outputs: ``tests/golden/*.npz`` (data only).
"""
from __future__ import annotations

import os
import random
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
REF_SRC = "/root/reference/src"

import oracle  # noqa: E402  (CPU restatement, used only as the stubbed BP)
from qldpc_fault_tolerance_amd import codes  # noqa: E402


class OracleBP:
    """Stand-in for ``ldpc.bp_decoder`` recording how the reference constructs it."""

    log = []

    def __init__(self, parity_check_matrix=None, channel_probs=None, max_iter=0, bp_method="minimum_sum",
                 ms_scaling_factor=1.0, **kw):
        if parity_check_matrix is None:
            parity_check_matrix = kw.pop("H")
        self.H = np.asarray(parity_check_matrix)
        self.channel_probs = np.asarray(channel_probs, dtype=np.float64)
        self.max_iter_arg = max_iter
        self.max_iter = int(max_iter)  # Cython int conversion truncates (quirk Q1)
        self.bp_method = bp_method
        self.alpha = ms_scaling_factor
        OracleBP.log.append(dict(shape=self.H.shape, max_iter_arg=float(max_iter), bp_method=bp_method,
                                 alpha=float(ms_scaling_factor), probs=self.channel_probs.copy()))

    def decode(self, synd):
        if not hasattr(self, "_csr"):  # converted once per decoder object (dense H -> CSR)
            self._csr = codes.CSR.from_dense(self.H)
        corr, _, _ = oracle.bp_decode_batch(self._csr, self.channel_probs, self.max_iter, self.bp_method, self.alpha,
                                            np.asarray(synd).reshape(1, -1), 64, nthreads=1)
        return corr[0].astype(int)


def install_stubs():
    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    class _Anything:
        def __init__(self, *a, **k):
            raise RuntimeError("stubbed third-party class used")

    mod("graph_tools", Graph=_Anything)
    ldpc = mod("ldpc", bp_decoder=OracleBP)
    ldpc.codes = mod("ldpc.codes")
    ldpc.code_util = mod("ldpc.code_util", compute_code_distance=lambda H: 0)
    ldpc.mod2 = mod("ldpc.mod2")
    bposd = mod("bposd", bposd_decoder=_Anything)
    bposd.css_decode_sim = mod("bposd.css_decode_sim", css_decode_sim=_Anything)
    bposd.hgp = mod("bposd.hgp", hgp=_Anything)
    bposd.css = mod("bposd.css", css_code=_Anything)
    for name in ("stim", "pymatching", "sinter"):
        m = mod(name)
        m.__getattr__ = lambda attr: type(attr, (), {})  # annotation-only names (stim.Circuit, ...)
    import matplotlib

    matplotlib.use("Agg")
    sys.path.insert(0, REF_SRC)


def main():
    install_stubs()
    import Decoders  # noqa: F401
    import Decoders_SpaceTime
    import Simulators
    import Simulators_SpaceTime

    # serial parmap: same semantics, no fork (src/Simulators.py:45-61)
    Simulators.parmap = lambda f, X, nprocs=1: [f(x) for x in X]
    Simulators_SpaceTime.parmap = Simulators.parmap

    code = codes.get_code("hgp_34_n225")
    n = code.N
    out = {}

    # ---- A5: _generate_error on seeded CPython random, with the raw uniforms
    for tag, probs in [("dep05", [0.05 / 2] * 3), ("dep10", [0.10 / 2] * 3), ("asym", [0.03, 0.01, 0.07])]:
        sim = Simulators.CodeSimulator_DataError(code=code, decoder_x=None, decoder_z=None,
                                                 pauli_error_probs=probs, eval_logical_type="Total")
        E_x, E_z, U = [], [], []
        for s in range(20):
            random.seed(1000 + s)
            ex, ez = sim._generate_error()
            random.seed(1000 + s)
            U.append([random.random() for _ in range(n)])
            E_x.append(ex.copy())
            E_z.append(ez.copy())
        out[f"gen_{tag}_probs"] = np.array(probs)
        out[f"gen_{tag}_u"] = np.array(U)
        out[f"gen_{tag}_ex"] = np.array(E_x, dtype=np.uint8)
        out[f"gen_{tag}_ez"] = np.array(E_z, dtype=np.uint8)

    # ---- A1-A3, A6-A8: _single_run through the reference decoder factory
    for p in (0.03, 0.06):
        cls = Decoders.BP_Decoder_Class(max_iter_ratio=10, bp_method="minimum_sum", ms_scaling_factor=0.625)
        OracleBP.log.clear()
        dx = cls.GetDecoder({"h": code.hz, "p_data": p})
        dz = cls.GetDecoder({"h": code.hx, "p_data": p})
        out[f"factory_p{int(p*100)}_max_iter_arg"] = np.array([d["max_iter_arg"] for d in OracleBP.log])
        out[f"factory_p{int(p*100)}_probs"] = np.array([d["probs"] for d in OracleBP.log])
        probs = [p / 2] * 3  # EvalWER data branch (src/Simulators.py:763-764)
        for mode in ("X", "Z", "Total"):
            sim = Simulators.CodeSimulator_DataError(code=code, decoder_x=dx, decoder_z=dz,
                                                     pauli_error_probs=probs, eval_logical_type=mode)
            flags = []
            for s in range(60):
                random.seed(5000 + s)
                flags.append(int(sim._single_run()))
            out[f"run_p{int(p*100)}_{mode}_fail"] = np.array(flags, dtype=np.uint8)
        # the uniforms of those shots (same seeds), for replay through the engine
        U = []
        for s in range(60):
            random.seed(5000 + s)
            U.append([random.random() for _ in range(n)])
        out[f"run_p{int(p*100)}_u"] = np.array(U)

    # ---- A8: WordErrorRate formula incl. quirk Q2, with injected failure lists
    class _K:
        N, K = n, code.K
        hx, hz, lx, lz = code.hx, code.hz, code.lx, code.lz

    wer_cases = []
    for num_run, nfail in [(1000, 0), (1000, 17), (5000, 1234), (200, 199), (10, 10)]:
        sim = Simulators.CodeSimulator_DataError(code=_K, decoder_x=None, decoder_z=None)
        flags = [1] * nfail + [0] * (num_run - nfail)
        sim._single_run = (lambda it=iter(flags): next(it))
        wer, eb = sim.WordErrorRate(num_run)
        wer_cases.append([num_run, nfail, wer, eb])
    out["wer_cases"] = np.array(wer_cases, dtype=np.float64)

    # ---- A10: GetSpaceTimeCheckMat
    for t0 in (1, 2, 3):
        ST = Decoders_SpaceTime.GetSpaceTimeCheckMat(code.hx.astype(float), t0)
        c = codes.CSR.from_dense(ST)
        out[f"st_t{t0}_shape"] = np.array(ST.shape)
        out[f"st_t{t0}_row_ptr"] = c.row_ptr
        out[f"st_t{t0}_col_idx"] = c.col_idx

    # ---- A11/A12: ST decoder factory + decode fold on random detector histories
    stc = Decoders_SpaceTime.ST_BP_Decoder_Class(max_iter_ratio=10, bp_method="minimum_sum", ms_scaling_factor=0.625)
    OracleBP.log.clear()
    st_dec = stc.GetDecoder({"h": code.hz, "p_data": 0.02, "p_syndrome": 0.02, "num_rep": 3})
    out["stfactory_max_iter_arg"] = np.array([OracleBP.log[0]["max_iter_arg"]])
    out["stfactory_probs"] = OracleBP.log[0]["probs"]
    rng = np.random.default_rng(3)
    hist = (rng.random((10, 3, code.hz.shape[0])) < 0.03).astype(np.float64)
    out["stdec_hist"] = hist.astype(np.uint8)
    out["stdec_corr"] = np.array([st_dec.decode(h) for h in hist], dtype=np.uint8)

    # ---- A13: CodeSimulator_Phenon_SpaceTime detector histories (quirk Q3) and failures
    class Capture:
        def __init__(self, inner):
            self.inner, self.seen = inner, []

        def decode(self, x):
            self.seen.append(np.array(x, dtype=np.uint8))
            return self.inner.decode(x)

    p = 0.02
    d1x = Capture(stc.GetDecoder({"h": code.hz, "p_data": p, "p_syndrome": p, "num_rep": 3}))
    d1z = Capture(stc.GetDecoder({"h": code.hx, "p_data": p, "p_syndrome": p, "num_rep": 3}))
    cls = Decoders.BP_Decoder_Class(max_iter_ratio=10, bp_method="minimum_sum", ms_scaling_factor=0.625)
    d2x = Capture(cls.GetDecoder({"h": code.hz, "p_data": p}))
    d2z = Capture(cls.GetDecoder({"h": code.hx, "p_data": p}))
    sim = Simulators_SpaceTime.CodeSimulator_Phenon_SpaceTime(
        code=code, decoder1_x=d1x, decoder1_z=d1z, decoder2_x=d2x, decoder2_z=d2z,
        pauli_error_probs=[p / 2] * 3, q=p, eval_logical_type="Total", num_rep=3)
    flags, U = [], []
    n_u = 2 * (3 * (n + code.hx.shape[0] + code.hz.shape[0])) + (n + code.hx.shape[0] + code.hz.shape[0])
    for s in range(12):
        random.seed(9000 + s)
        flags.append(int(sim._single_run(3)))  # num_rounds = 3 -> 2 noisy rounds of 3 reps + final
        random.seed(9000 + s)
        U.append([random.random() for _ in range(n_u)])
    out["phenst_fail"] = np.array(flags, dtype=np.uint8)
    out["phenst_u"] = np.array(U)
    out["phenst_d1z_hist"] = np.array(d1z.seen)
    out["phenst_d1x_hist"] = np.array(d1x.seen)
    out["phenst_d2z_synd"] = np.array(d2z.seen)
    out["phenst_d2x_synd"] = np.array(d2x.seen)
    # WordErrorRate formula of the ST simulator (:531-548) with injected flags
    st_wer = []
    for num_cycles, num_samples, nfail in [(7, 100, 9), (13, 400, 77), (13, 50, 50)]:
        sim2 = Simulators_SpaceTime.CodeSimulator_Phenon_SpaceTime(
            code=_K, decoder1_x=None, decoder1_z=None, decoder2_x=None, decoder2_z=None,
            pauli_error_probs=[p / 2] * 3, q=p, eval_logical_type="Total", num_rep=3)
        fl = [1] * nfail + [0] * (num_samples - nfail)
        sim2._single_run = (lambda num_rounds, it=iter(fl): next(it))
        w, _ = sim2.WordErrorRate(num_cycles, num_samples)
        st_wer.append([num_cycles, num_samples, nfail, w])
    out["phenst_wer_cases"] = np.array(st_wer, dtype=np.float64)

    np.savez_compressed(os.path.join(HERE, "reference_harness_n225.npz"), **out)
    print("wrote", os.path.join(HERE, "reference_harness_n225.npz"), len(out), "arrays")


def main_phen():
    """Single-shot phenomenological simulator (CodeSimulator_Phenon, src/Simulators.py:189-381) and
    FirstMinBPDecoder (src/Decoders.py:49-74) -> tests/golden/reference_harness_phen_n225.npz."""
    install_stubs()
    import Decoders
    import Simulators

    Simulators.parmap = lambda f, X, nprocs=1: [f(x) for x in X]
    code = codes.get_code("hgp_34_n225")
    n, mx, mz = code.N, code.hx.shape[0], code.hz.shape[0]
    out = {}

    class Capture:
        def __init__(self, inner):
            self.inner, self.seen = inner, []

        def decode(self, x):
            self.seen.append(np.array(x, dtype=np.uint8))
            return self.inner.decode(x)

    p = 0.02
    cls = Decoders.BP_Decoder_Class(max_iter_ratio=10, bp_method="minimum_sum", ms_scaling_factor=0.625)
    hx_ext = np.hstack([code.hx, np.identity(mx)])
    hz_ext = np.hstack([code.hz, np.identity(mz)])
    d1x = Capture(cls.GetDecoder({"h": hz_ext, "p_data": p, "p_syndrome": p}))
    d1z = Capture(cls.GetDecoder({"h": hx_ext, "p_data": p, "p_syndrome": p}))
    d2x = Capture(cls.GetDecoder({"h": code.hz, "p_data": p}))
    d2z = Capture(cls.GetDecoder({"h": code.hx, "p_data": p}))
    out["phen_factory_max_iter_arg"] = np.array([d1x.inner.max_iter, d2x.inner.max_iter], dtype=np.float64)
    sim = Simulators.CodeSimulator_Phenon(code=code, decoder1_x=d1x, decoder1_z=d1z, decoder2_x=d2x,
                                          decoder2_z=d2z, pauli_error_probs=[p / 2] * 3, q=p,
                                          eval_logical_type="Total")
    num_rounds = 3
    n_u = num_rounds * (n + mx + mz)
    flags, U = [], []
    for s in range(16):
        random.seed(7000 + s)
        flags.append(int(sim._single_run(num_rounds)))
        random.seed(7000 + s)
        U.append([random.random() for _ in range(n_u)])
    out["phen_fail"] = np.array(flags, dtype=np.uint8)
    out["phen_u"] = np.array(U)
    out["phen_d1z_synd"] = np.array(d1z.seen)
    out["phen_d1x_synd"] = np.array(d1x.seen)
    out["phen_d2z_synd"] = np.array(d2z.seen)
    out["phen_d2x_synd"] = np.array(d2x.seen)
    # WordErrorRate / WordErrorProbability formulas (:329-381) on injected failure counts
    cases = []
    for num_rounds_, num_samples, nfail in [(3, 100, 9), (5, 400, 77), (1, 50, 50)]:
        sim2 = Simulators.CodeSimulator_Phenon(code=code, pauli_error_probs=[p / 2] * 3, q=p)
        for fn in ("WordErrorRate", "WordErrorProbability"):
            fl = [1] * nfail + [0] * (num_samples - nfail)
            sim2._single_run = (lambda num_rounds, it=iter(fl): next(it))
            w, eb = getattr(sim2, fn)(num_rounds_, num_samples)
            cases.append([num_rounds_, num_samples, nfail, 0 if fn == "WordErrorRate" else 1, w,
                          np.nan if eb is None else eb])
    out["phen_wer_cases"] = np.array(cases, dtype=np.float64)
    # FirstMinBPDecoder: repeated max_iter=1 BP with the syndrome-weight stopping rule
    rng = np.random.default_rng(11)
    fm = Decoders.FirstMinBPDecoder(hz_ext, np.hstack([p * np.ones(n), p * np.ones(mz)]), 20, "minimum_sum", 0.625)
    S = (rng.random((24, mz)) < 0.06).astype(np.uint8)
    out["firstmin_synd"] = S
    out["firstmin_corr"] = np.array([fm.decode(s.astype(float)) for s in S], dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, "reference_harness_phen_n225.npz"), **out)
    print("wrote", os.path.join(HERE, "reference_harness_phen_n225.npz"), len(out), "arrays")


CONFIG_CODES = ["hgp_34_n1600", "LP_Matg8_L30_Dmin20", "GenBicycleA1", "GenBicycleA2", "GenBicycleA3", "GenBicycleA4"]


def main_configs():
    """Harness goldens on the BASELINE config codes -> tests/golden/reference_harness_configs.npz.

    For each data-error config code (the synthesized [[1600,64]] HGP stand-in, the reference's own
    LP_Matg8_L30_Dmin20 and GenBicycleA1-A4 matrices): ``_generate_error`` outputs and
    ``_single_run`` failure flags (X / Z / Total) of the reference's CodeSimulator_DataError with the
    reference's BP_Decoder_Class (BP = the oracle stub), and for config 5 (hgp_34_n1225_q3 stand-in,
    num_rep = 3) the detector histories, final syndromes and failures of
    CodeSimulator_Phenon_SpaceTime._single_run.  Uniforms are NOT stored: each shot re-seeds CPython's
    ``random`` (seed recorded), so a test regenerates the identical stream.  Bits are packed
    (np.packbits along the last axis).
    """
    install_stubs()
    import Decoders
    import Decoders_SpaceTime
    import Simulators
    import Simulators_SpaceTime

    Simulators.parmap = lambda f, X, nprocs=1: [f(x) for x in X]
    out = {}
    cls = Decoders.BP_Decoder_Class(max_iter_ratio=10, bp_method="minimum_sum", ms_scaling_factor=0.625)
    for name in CONFIG_CODES:
        code = codes.get_code(name)
        n = code.N
        tag = name
        # ---- A5: _generate_error at [p/2]*3 (p = 0.08) and an asymmetric split
        for gtag, probs in (("dep08", [0.04] * 3), ("asym", [0.03, 0.01, 0.07])):
            E_x, E_z = [], []
            sim = Simulators.CodeSimulator_DataError(code=code, decoder_x=None, decoder_z=None,
                                                     pauli_error_probs=probs, eval_logical_type="Total")
            for s in range(8):
                random.seed(31000 + s)
                ex, ez = sim._generate_error()
                E_x.append(ex.copy())
                E_z.append(ez.copy())
            out[f"{tag}_gen_{gtag}_probs"] = np.array(probs)
            out[f"{tag}_gen_{gtag}_seed0"] = np.array([31000])
            out[f"{tag}_gen_{gtag}_ex"] = np.packbits(np.array(E_x, dtype=np.uint8), axis=-1)
            out[f"{tag}_gen_{gtag}_ez"] = np.packbits(np.array(E_z, dtype=np.uint8), axis=-1)
        # ---- A1-A3, A6-A8: _single_run with the reference decoder factory (EvalWER data branch)
        S = 500  # shots per (code, p): >= 500 (VERDICT r02 asked for thicker fixtures)
        for p in (0.04, 0.08):
            dx = cls.GetDecoder({"h": code.hz, "p_data": p})
            dz = cls.GetDecoder({"h": code.hx, "p_data": p})
            for mode in ("X", "Z", "Total"):
                sim = Simulators.CodeSimulator_DataError(code=code, decoder_x=dx, decoder_z=dz,
                                                         pauli_error_probs=[p / 2] * 3, eval_logical_type=mode)
                flags = []
                for s in range(S):
                    random.seed(41000 + s)
                    flags.append(int(sim._single_run()))
                out[f"{tag}_run_p{int(round(p * 100))}_{mode}_fail"] = np.array(flags, dtype=np.uint8)
            out[f"{tag}_run_p{int(round(p * 100))}_seed0"] = np.array([41000])
        print(name, "done", flush=True)

    # ---- config 5: CodeSimulator_Phenon_SpaceTime on the 1764 x 5439 space-time graph
    class Capture:
        def __init__(self, inner):
            self.inner, self.seen = inner, []

        def decode(self, x):
            self.seen.append(np.array(x, dtype=np.uint8))
            return self.inner.decode(x)

    code = codes.get_code("hgp_34_n1225_q3")
    p = 0.01
    stc = Decoders_SpaceTime.ST_BP_Decoder_Class(max_iter_ratio=10, bp_method="minimum_sum", ms_scaling_factor=0.625)
    d1x = Capture(stc.GetDecoder({"h": code.hz, "p_data": p, "p_syndrome": p, "num_rep": 3}))
    d1z = Capture(stc.GetDecoder({"h": code.hx, "p_data": p, "p_syndrome": p, "num_rep": 3}))
    d2x = Capture(cls.GetDecoder({"h": code.hz, "p_data": p}))
    d2z = Capture(cls.GetDecoder({"h": code.hx, "p_data": p}))
    sim = Simulators_SpaceTime.CodeSimulator_Phenon_SpaceTime(
        code=code, decoder1_x=d1x, decoder1_z=d1z, decoder2_x=d2x, decoder2_z=d2z,
        pauli_error_probs=[p / 2] * 3, q=p, eval_logical_type="Total", num_rep=3)
    flags = []
    for s in range(100):
        random.seed(51000 + s)
        flags.append(int(sim._single_run(3)))  # 2 noisy rounds of 3 repetitions + the perfect round
    out["st1225_seed0"] = np.array([51000])
    out["st1225_fail"] = np.array(flags, dtype=np.uint8)
    out["st1225_d1z_hist"] = np.packbits(np.array(d1z.seen), axis=-1)
    out["st1225_d1x_hist"] = np.packbits(np.array(d1x.seen), axis=-1)
    out["st1225_d2z_synd"] = np.packbits(np.array(d2z.seen), axis=-1)
    out["st1225_d2x_synd"] = np.packbits(np.array(d2x.seen), axis=-1)
    path = os.path.join(HERE, "reference_harness_configs.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, len(out), "arrays")


def main_fits():
    """Threshold tooling -> tests/golden/reference_fits.npz.

    Runs the reference's own fit functions (src/Simulators.py:675-741, 912-963;
    src/Simulators_SpaceTime.py:1080-1149, 1311-1362) on fixed injected WER arrays: DistanceEst,
    ThresholdEst_extrapolation, and CodeFamily{,_SpaceTime}.EvalThreshold / EvalSustainableThreshold /
    EvalEffectiveDistances with EvalWER / EvalThreshold replaced by recorders returning the injected
    data (the p grids they were called with are recorded too).
    """
    install_stubs()
    import Simulators
    import Simulators_SpaceTime
    import matplotlib.pyplot as plt

    plt.show = lambda *a, **k: None
    out = {}
    rng = np.random.default_rng(123)
    d_true = np.array([4.0, 6.0, 8.0])
    pc_true, A_true = 0.08, 0.3
    # WER arrays [codes x p] from the extrapolation model, with 3 % multiplicative noise
    p_thr = 10 ** np.linspace(np.log10(0.08 * 0.4), np.log10(0.08 * 0.8), 6)
    wer_thr = np.array([A_true * (p_thr / pc_true) ** (d / 2) for d in d_true]) * (1 + 0.03 * rng.standard_normal((3, 6)))
    p_dist = 10 ** np.linspace(np.log10(0.08 / 6), np.log10(0.08 / 4), 5)
    wer_dist = np.array([0.5 * p_dist ** (d / 2) for d in d_true]) * (1 + 0.03 * rng.standard_normal((3, 5)))
    out["thr_p"], out["thr_wer"], out["dist_p"], out["dist_wer"] = p_thr, wer_thr, p_dist, wer_dist
    for mod, tag in ((Simulators, "sim"), (Simulators_SpaceTime, "st")):
        out[f"{tag}_distance_est"] = np.array(mod.DistanceEst(p_thr, wer_thr))
        out[f"{tag}_threshold_extrap"] = np.array([mod.ThresholdEst_extrapolation(p_thr, wer_thr)])
    # CodeFamily.EvalThreshold / EvalEffectiveDistances with a recording EvalWER
    seen = []

    def rec_evalwer(data):
        def f(self, noise_model, eval_logical_type, eval_p_list, *a, **k):
            seen.append(np.array(eval_p_list, dtype=np.float64))
            return data
        return f

    fam = Simulators.CodeFamily([], None, None)
    Simulators.CodeFamily.EvalWER = rec_evalwer(wer_thr)
    out["fam_eval_threshold"] = np.array([fam.EvalThreshold("data", "Total", "extrapolation", 0.08, 100)])
    out["fam_eval_threshold_p"] = seen[-1]
    Simulators.CodeFamily.EvalWER = rec_evalwer(wer_dist)
    out["fam_eval_distances"] = np.array(fam.EvalEffectiveDistances("data", "Total", "extrapolation", 0.08, 100))
    out["fam_eval_distances_p"] = seen[-1]
    # EvalSustainableThreshold: EvalThreshold replaced by thresholds that saturate with the cycle count
    cycles = np.array([1, 3, 5, 9, 15, 25])
    thr = 0.03 * (1 - (1 - 0.06 / 0.03) * np.exp(-0.2 * cycles)) * (1 + 0.01 * rng.standard_normal(6))
    calls = []

    def rec_thr(self, noise_model, eval_logical_type, eval_method, est_threshold, num_samples, num_cycles=1, **k):
        calls.append([num_samples, num_cycles])
        return float(thr[list(cycles).index(num_cycles)])

    out["sus_cycles"], out["sus_thr"] = cycles, thr
    Simulators.CodeFamily.EvalThreshold = rec_thr
    out["fam_sus"] = np.array([fam.EvalSustainableThreshold("phenl", "Total", "extrapolation", 0.05, 12000,
                                                             list(cycles))])
    out["fam_sus_calls"] = np.array(calls)
    calls.clear()
    stfam = Simulators_SpaceTime.CodeFamily_SpaceTime([], None, None)
    Simulators_SpaceTime.CodeFamily_SpaceTime.EvalThreshold = rec_thr
    out["st_sus"] = np.array([stfam.EvalSustainableThreshold("phenl", "Total", "extrapolation", 0.05, 12000,
                                                              list(cycles))])
    out["st_sus_calls"] = np.array(calls)
    Simulators_SpaceTime.CodeFamily_SpaceTime.EvalWER = rec_evalwer(wer_dist)
    out["st_eval_distances"] = np.array(stfam.EvalEffectiveDistances("phenl", "Total", "extrapolation", 0.08, 100))
    out["st_eval_distances_p"] = seen[-1]
    path = os.path.join(HERE, "reference_fits.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, len(out), "arrays")


def main_notebook():
    """The Threshold notebook's own fit (``.ipynb_checkpoints/Threshold-checkpoint.ipynb`` cells 1-2:
    ``FitDistance`` / ``EmpericalFit`` / ``ThresholdEst``, lines 33-120) -> tests/golden/notebook_fits.npz.

    The two cells' source is executed as the notebook did (no plot), on fixed WER arrays over the
    p grids of cells 16 and 25: inputs and the returned ``(A, p_c)`` are stored, to pin the
    restatement in tests/notebook_pin.py that the threshold pin (tests/test_gpu_notebook_pin.py) uses.
    """
    import contextlib
    import copy
    import io
    import json

    import matplotlib.pyplot as plt
    from scipy.optimize import curve_fit

    nb = json.load(open(os.path.join(os.path.dirname(REF_SRC), ".ipynb_checkpoints", "Threshold-checkpoint.ipynb")))
    ns = {"np": np, "copy": copy, "plt": plt, "curve_fit": curve_fit}
    for c in (1, 2):
        exec("".join(nb["cells"][c]["source"]), ns)
    rng = np.random.default_rng(2024)
    out = {}
    grids = {"lp": np.linspace(2e-2, 3.5e-2, 6), "toric": np.linspace(0.8e-2, 2e-2, 6)}
    k = 0
    for gname, P in grids.items():
        for d, pc, A in (((6, 8, 10), 0.05, 0.02), ((3, 5, 7), 0.03, 0.05), ((2, 3, 4), 0.06, 0.1)):
            for noise in (0.0, 0.1, 0.3):
                wer = np.array([A * (P / pc) ** (dd / 2) for dd in d]) * (1 + noise * rng.standard_normal((3, 6)))
                wer = np.abs(wer)
                buf = io.StringIO()
                try:
                    with contextlib.redirect_stdout(buf):  # ThresholdEst returns p_c and prints "A: .. p_c: .."
                        pc_fit = ns["ThresholdEst"](P, wer, False)
                    words = buf.getvalue().split()
                    res = np.array([float(words[words.index("A:") + 1]), float(pc_fit)])
                except Exception:  # noqa: BLE001
                    res = np.array([np.nan, np.nan])
                out[f"case{k}_p"], out[f"case{k}_wer"], out[f"case{k}_A_pc"] = P, wer, res
                k += 1
    out["ncases"] = np.array([k])
    path = os.path.join(HERE, "notebook_fits.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, k, "cases")


def schedule_cases():
    """(name, H) of the CX-schedule fixtures: the demo's d3 toric code, the d3 surface code of the
    Threshold notebook (ring codes without their last row), hgp_34_n225 and GenBicycleA1."""
    def ring(d):
        h = np.zeros((d, d), np.uint8)
        for i in range(d):
            h[i, i] = h[i, (i + 1) % d] = 1
        return h

    tor = codes.hgp(ring(3), ring(3))
    sur = codes.hgp(ring(3)[:-1, :], ring(3)[:-1, :])
    n225 = codes.get_code("hgp_34_n225")
    gbc = codes.get_code("GenBicycleA1")
    return [("toric3_hx", tor.hx), ("toric3_hz", tor.hz), ("surface3_hx", sur.hx), ("surface3_hz", sur.hz),
            ("n225_hx", n225.hx), ("n225_hz", n225.hz), ("gbcA1_hx", gbc.hx)]


def main_schedules():
    """ColorationCircuit / RandomCircuit (src/CircuitScheduling.py) of the reference itself: it imports
    only numpy and networkx, both present, so no stub is needed."""
    sys.path.insert(0, REF_SRC)
    import CircuitScheduling as CS  # noqa: E402  (the reference's own module)

    out = {}
    for name, H in schedule_cases():
        for kind, fn in (("color", CS.ColorationCircuit), ("random", CS.RandomCircuit)):
            sched = fn(np.asarray(H).astype(int))
            keys, vals, offs = [], [], [0]
            for step in sched:
                for k in step:  # insertion order kept
                    keys.append(int(k))
                    vals.append(int(step[k]))
                offs.append(len(keys))
            out[f"{name}_{kind}_keys"] = np.array(keys, np.int32)
            out[f"{name}_{kind}_vals"] = np.array(vals, np.int32)
            out[f"{name}_{kind}_offs"] = np.array(offs, np.int32)
    path = os.path.join(HERE, "reference_circuit_schedules.npz")
    np.savez_compressed(path, **out)
    print("wrote", path)


class _RecTarget:
    """``stim.target_rec(k)``."""

    def __init__(self, k):
        self.k = int(k)


# gates that never fuse with a neighbour in stim (annotations); every other gate fuses with an
# immediately preceding instruction of the same gate and arguments (stim's append / parse / +=)
_STIM_NOFUSE = {"DETECTOR", "OBSERVABLE_INCLUDE", "SHIFT_COORDS", "TICK"}
_DEM_STYLE = ["exact"]


class RecordingCircuit:
    """A recording stand-in for ``stim.Circuit`` (stim is absent): it keeps the instructions the
    reference's ``_generate_circuit`` appends (gate, targets, arguments; consecutive same-gate
    same-argument instructions fused, as stim does), renders them as stim circuit text for
    ``AddCXError`` (``src/ErrorPlugin.py:11-25``, which rewrites ``str(circuit)``) and parses that
    text back.  ``detector_error_model`` is the ONE place the engine enters: the recorded op list is
    handed to ``qldpc_fault_tolerance_amd.circuit.detector_error_model`` and rendered as DEM text
    (``_DEM_STYLE``), which the reference's own ``GenFaultHyperGraph`` / ``GenCorrecHyperGraph`` then
    parse unchanged."""

    def __init__(self, text=None):
        self.ops = []  # [name, targets (int qubit | _RecTarget), args tuple]
        if text is not None:
            for line in str(text).split("\n"):
                line = line.strip()
                if not line or line in ("{", "}"):
                    continue
                head, _, rest = line.partition(" ")
                if "(" in head:
                    name = head[:head.index("(")]
                    args = tuple(float(a) for a in head[head.index("(") + 1:head.rindex(")")].split(","))
                else:
                    name, args = head, ()
                tg = [(_RecTarget(int(t[4:-1])) if t.startswith("rec[") else int(t)) for t in rest.split()]
                self._push(name, tg, args)

    def _push(self, name, targets, args):
        name = name.upper()
        last = self.ops[-1] if self.ops else None
        if last is not None and name not in _STIM_NOFUSE and last[0] == name and last[2] == args:
            last[1].extend(targets)
        else:
            self.ops.append([name, list(targets), args])

    def append(self, name, targets=(), arg=None):
        if arg is None:
            args = ()
        elif isinstance(arg, (list, tuple)):
            args = tuple(float(a) for a in arg)
        else:
            args = (float(arg),)
        tg = [t if isinstance(t, _RecTarget) else int(t) for t in (targets if len(targets) else [])]
        self._push(name, tg, args)

    def __add__(self, other):
        c = RecordingCircuit()
        for o in self.ops + other.ops:
            c._push(o[0], list(o[1]), o[2])
        return c

    def __mul__(self, k):
        c = RecordingCircuit()
        for _ in range(int(k)):
            for o in self.ops:
                c.ops.append([o[0], list(o[1]), o[2]])  # flattened REPEAT: no fusion across copies
        return c

    __rmul__ = __mul__

    def __str__(self):
        lines = []
        for name, tg, args in self.ops:
            a = "(" + ", ".join(repr(x) for x in args) + ")" if args else ""
            t = " ".join(f"rec[{x.k}]" if isinstance(x, _RecTarget) else str(x) for x in tg)
            lines.append(f"{name}{a} {t}".rstrip())
        return "\n".join(lines) + "\n"

    def engine_circuit(self):
        from qldpc_fault_tolerance_amd import circuit as C

        return C.StimCircuit([C.Op(n, [(x.k if isinstance(x, _RecTarget) else x) for x in tg],
                                   (args[0] if args else None)) for n, tg, args in self.ops])

    def detector_error_model(self, flatten_loops=True):
        text = self.engine_circuit().detector_error_model().to_text(_DEM_STYLE[0])

        class _Dem:
            def __str__(self):
                return text

        return _Dem()

    def compile_detector_sampler(self):
        return None


def circuit_cases():
    """(tag, code, p, error_params, num_cycles, num_rep, circuit_type) of the circuit fixtures: the
    demo (SpaceTimeDecodingDemo.ipynb cell 2), every noise source at the GPU tests' rate with both
    schedules, distinct rates per source, and a low rate whose mechanisms stim prints in exponent
    notation (the reference's regex reads their mantissas)."""
    def ring(d):
        h = np.zeros((d, d), np.uint8)
        for i in range(d):
            h[i, i] = h[i, (i + 1) % d] = 1
        return h

    tor = codes.hgp(ring(3), ring(3))
    allp = lambda p: {"p_i": p, "p_state_p": p, "p_m": p, "p_CX": p, "p_idling_gate": p}  # noqa: E731
    return [
        ("demo", tor, 1e-3, {"p_i": 0.0, "p_state_p": 0.0, "p_m": 0.0, "p_CX": 1e-3, "p_idling_gate": 0.0}, 13, 3,
         "coloration"),
        ("all3c", tor, 3e-3, allp(3e-3), 13, 3, "coloration"),
        ("all3r", tor, 3e-3, allp(3e-3), 13, 3, "random"),
        ("mixed", tor, 6e-3, {"p_i": 2e-3, "p_state_p": 3e-3, "p_m": 4e-3, "p_CX": 5e-3, "p_idling_gate": 1e-3}, 5, 2,
         "random"),
        ("low", tor, 5e-5, allp(5e-5), 7, 3, "coloration"),
    ]


def _pack_ops(ops):
    names = np.array([o[0] for o in ops], dtype="<U20")
    args = np.array([(o[2][0] if o[2] else np.nan) for o in ops], dtype=np.float64)
    offs = np.cumsum([0] + [len(o[1]) for o in ops]).astype(np.int64)
    tg = np.array([(x.k if isinstance(x, _RecTarget) else x) for o in ops for x in o[1]], dtype=np.int64)
    return names, args, offs, tg


def main_circuit():
    """Circuit-level fixtures from the reference's own ``CodeSimulator_Circuit_SpaceTime``
    (``src/Simulators_SpaceTime.py:672-967``) -> tests/golden/reference_circuit.npz.

    With the stubs of :func:`install_stubs` plus :class:`RecordingCircuit` as ``stim.Circuit``, the
    reference's ``_generate_circuit`` (:737-940) and ``AddCXError`` run unchanged; the recorded op
    lists of ``circuit`` / ``fault_circuit`` are stored.  Its ``_generate_circuit_graph`` (:943-967)
    then runs unchanged on the engine's DEM of the recorded fault circuit, rendered as DEM text twice:
    ``exact`` (the engine's mechanism order, round-trip probabilities) and ``stim`` (stim's order and
    6-significant-digit ``%g`` probabilities, which its regex parse reads back).  Stored: h1, L1,
    channel_ps1, h2, L2, channel_ps2, h1_space_cor of both."""
    install_stubs()
    stim = sys.modules["stim"]
    stim.Circuit = RecordingCircuit
    stim.target_rec = _RecTarget
    import Simulators_SpaceTime as SST

    out = {}
    for tag, code, p, ep, ncyc, nrep, ctype in circuit_cases():
        sim = SST.CodeSimulator_Circuit_SpaceTime(code=code, p=p, num_cycles=ncyc, num_rep=nrep, error_params=dict(ep),
                                                  eval_logical_type="Z", circuit_type=ctype)
        sim._generate_circuit()
        for which, circ in (("circuit", sim.circuit), ("fault", sim.fault_circuit)):
            names, args, offs, tg = _pack_ops(circ.ops)
            out[f"{tag}_{which}_names"], out[f"{tag}_{which}_args"] = names, args
            out[f"{tag}_{which}_offs"], out[f"{tag}_{which}_targets"] = offs, tg
        for style in ("exact", "stim"):
            _DEM_STYLE[0] = style
            sim._generate_circuit_graph()
            g = sim.circuit_graph
            for k in ("h1", "L1", "h2", "L2"):
                out[f"{tag}_{style}_{k}"] = np.asarray(g[k], dtype=np.uint8)
            for k in ("channel_ps1", "channel_ps2"):
                out[f"{tag}_{style}_{k}"] = np.asarray(g[k], dtype=np.float64)
            out[f"{tag}_{style}_h1_space_cor"] = np.asarray(sim.h1_space_cor, dtype=np.uint8)
        out[f"{tag}_params"] = np.array([p, ep["p_i"], ep["p_state_p"], ep["p_m"], ep["p_CX"], ep["p_idling_gate"], ncyc,
                                         nrep, ctype == "random"], dtype=np.float64)
        print(tag, "h1", out[f"{tag}_exact_h1"].shape, "h2", out[f"{tag}_exact_h2"].shape, flush=True)
    path = os.path.join(HERE, "reference_circuit.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, len(out), "arrays")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "circuit":
        main_circuit()
    elif len(sys.argv) > 1 and sys.argv[1] == "schedules":
        main_schedules()
    elif len(sys.argv) > 1 and sys.argv[1] == "notebook":
        main_notebook()
    elif len(sys.argv) > 1 and sys.argv[1] == "phen":
        main_phen()
    elif len(sys.argv) > 1 and sys.argv[1] == "configs":
        main_configs()
    elif len(sys.argv) > 1 and sys.argv[1] == "fits":
        main_fits()
    else:
        main()
