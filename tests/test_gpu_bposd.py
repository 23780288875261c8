"""GPU parity of BP+OSD (src/Decoders.py:26-41, :100-138).

Soft-output BP (engine 1 with posteriors, qldpc_bp_decode_batch_soft) must
match the oracle's min-sum bit-for-bit: corrections, iterations, convergence
and the final log_prob_ratios (fp64 = reference arithmetic; fp32 = the
oracle's fp32 mode).  BPOSD_Decoder (GPU BP -> native OSD) must then equal
the oracle's BP followed by its literal OSD restatement.
"""
import numpy as np
import pytest

from qldpc_fault_tolerance_amd import codes

pytestmark = pytest.mark.gpu


def _sample(H, p, B, seed):
    rng = np.random.default_rng(seed)
    e = (rng.random((B, H.shape[1])) < p).astype(np.uint8)
    return (e.astype(np.int64) @ H.T.astype(np.int64) % 2).astype(np.uint8), e


@pytest.mark.parametrize("precision", [64, 32])
@pytest.mark.parametrize("name", ["hgp_34_n225", "hgp_34_n1600", "LP_Matg8_L30_Dmin20"])
def test_soft_bp_posteriors_match_oracle(gpu, oracle, precision, name):
    from qldpc_fault_tolerance_amd.engine import DeviceBP

    code = codes.get_code(name)
    H = code.hz
    n = code.N
    mi = int(n / 10)
    p = 0.07
    synd, _ = _sample(H, p, 256, seed=precision + n)
    dec = DeviceBP(H, p, max_iter=mi, ms_scaling_factor=0.625, precision=precision, soft=True)
    assert dec.geometry()["engine"] == 1
    corr, iters, conv, post = dec.decode_batch_soft(synd)
    oc, oi, ov, op = oracle.bp_decode_batch_soft(H, p, mi, 0.625, synd, precision)
    assert np.array_equal(iters, oi) and np.array_equal(conv, ov)
    assert np.array_equal(corr, oc.astype(np.int64))
    assert np.array_equal(post, op)  # bit-exact posteriors
    # the soft path decodes like the default engine
    c2, i2, v2 = DeviceBP(H, p, max_iter=mi, ms_scaling_factor=0.625, precision=precision).decode_batch(synd)
    assert np.array_equal(c2, corr) and np.array_equal(i2, iters)


@pytest.mark.parametrize("method,order", [("osd_e", 10), ("osd_cs", 8), ("osd_0", 0)])
def test_bposd_decoder_matches_oracle(gpu, oracle, method, order):
    from qldpc_fault_tolerance_amd.decoders import BPOSD_Decoder

    code = codes.get_code("hgp_34_n225")
    H = code.hz
    p = 0.09
    mi = int(code.N / 10)
    synd, _ = _sample(H, p, 64, seed=order)
    dec = BPOSD_Decoder(H, p * np.ones(code.N), mi, "minimum_sum", 0.625, method, order)
    ow = dec.decode_batch(synd)
    oc, _, ov, op = oracle.bp_decode_batch_soft(H, p, mi, 0.625, synd, 64)
    assert (~ov).sum() > 0
    for b in range(synd.shape[0]):
        if ov[b]:
            assert np.array_equal(ow[b], oc[b])
        else:
            _, rw = oracle.osd_decode(H, p * np.ones(code.N), synd[b], op[b], method, order)
            assert np.array_equal(ow[b], rw), b
        assert np.array_equal(H.astype(np.int64) @ ow[b] % 2, synd[b])
    # single-syndrome API of the reference: decode(synd) -> osdw_decoding
    one = dec.decode(synd[0])
    assert np.array_equal(one, ow[0]) and np.array_equal(dec.osdw_decoding, ow[0])


def test_bposd_factory_and_simulator(gpu):
    """BPOSD_Decoder_Class.GetDecoder -> CodeSimulator_DataError per-shot plugin path:
    BP+OSD never leaves a syndrome mismatch, so it fails no more often than BP."""
    import random

    from qldpc_fault_tolerance_amd.decoders import BP_Decoder_Class, BPOSD_Decoder_Class
    from qldpc_fault_tolerance_amd.simulators import CodeSimulator_DataError

    code = codes.get_code("hgp_34_n225")
    p = 0.06
    cls = BPOSD_Decoder_Class(max_iter_ratio=10, bp_method="minimum_sum", ms_scaling_factor=0.625,
                              osd_method="osd_e", osd_order=10)
    dx = cls.GetDecoder({"h": code.hz, "p_data": p})
    dz = cls.GetDecoder({"h": code.hx, "p_data": p})
    random.seed(1234)
    sim = CodeSimulator_DataError(code, dx, dz, [p / 2] * 3, "Total")
    fails_osd = sum(sim._single_run() for _ in range(150))
    bcls = BP_Decoder_Class(max_iter_ratio=10, bp_method="minimum_sum", ms_scaling_factor=0.625)
    random.seed(1234)
    sim_bp = CodeSimulator_DataError(code, bcls.GetDecoder({"h": code.hz, "p_data": p}),
                                     bcls.GetDecoder({"h": code.hx, "p_data": p}), [p / 2] * 3, "Total")
    fails_bp = sum(sim_bp._single_run() for _ in range(150))
    assert fails_osd <= fails_bp


def test_bposd_shot_loop_matches_oracle_per_shot(gpu, oracle):
    """CodeSimulator_DataError with BPOSD decoders: fused GPU MC + OSD on the
    non-converged shots.  Per shot and sector, the failure equals the oracle's
    BP (+ literal OSD when BP did not converge) on the same Philox errors; the
    same seed with plain BP decoders fails at least as often."""
    from qldpc_fault_tolerance_amd.decoders import BP_Decoder_Class, BPOSD_Decoder_Class
    from qldpc_fault_tolerance_amd.simulators import CodeSimulator_DataError, gf2_rows

    code = codes.get_code("hgp_34_n225")
    p, order, S = 0.08, 4, 160
    cls = BPOSD_Decoder_Class(10, "minimum_sum", 0.625, "osd_e", order)
    dx, dz = cls.GetDecoder({"h": code.hz, "p_data": p}), cls.GetDecoder({"h": code.hx, "p_data": p})
    sim = CodeSimulator_DataError(code, dx, dz, [p / 2] * 3, "Total", seed=77)
    fails, shots, osd_n = sim.bposd_counts(S, batch=64, keep_shots=True)
    assert shots == S and osd_n > 0
    err, sf = sim.last_shots
    assert err.shape == (S, code.N) and sf.shape == (S, 2)
    assert fails == int((sf[:, 0] | sf[:, 1]).sum())
    mi = int(code.N / 10)
    for q, H, L in ((0, code.hz, code.lz), (1, code.hx, code.lx)):
        e = ((err >> q) & 1).astype(np.uint8)
        synd = gf2_rows(code.csr("hz" if q == 0 else "hx"), e)
        oc, _, ov, op = oracle.bp_decode_batch_soft(H, p, mi, 0.625, synd, 64)
        for s in range(S):
            x = oc[s] if ov[s] else oracle.osd_decode(H, p * np.ones(code.N), synd[s], op[s], "osd_e", order)[1]
            r = (e[s] ^ x).astype(np.int64)
            f = bool((H.astype(np.int64) @ r % 2).any() or (L.astype(np.int64) @ r % 2).any())
            assert f == bool(sf[s, q]), (q, s)
    bcls = BP_Decoder_Class(10, "minimum_sum", 0.625)
    sim_bp = CodeSimulator_DataError(code, bcls.GetDecoder({"h": code.hz, "p_data": p}),
                                     bcls.GetDecoder({"h": code.hx, "p_data": p}), [p / 2] * 3, "Total", seed=77)
    assert sim_bp.fused_counts(S).failures >= fails
    # WordErrorRate routes BPOSD decoders through the same loop
    wer, _ = CodeSimulator_DataError(code, dx, dz, [p / 2] * 3, "Total", seed=77).WordErrorRate(S)
    from qldpc_fault_tolerance_amd.simulators import word_error_rate

    assert wer == word_error_rate(fails, S, code.K)[0]


# elimination modes of osd_gpu_kernel: the default (register rows for m <= 768 / 1024), the
# LDS-resident word-major image (QLDPC_OSD_RR=0) and the HBM slice (QLDPC_OSD_RR=0 QLDPC_OSD_LDS=0)
# and the opt-in panel eliminations of the register rows (QLDPC_OSD_PNL=1: one search wave; 2: every
# thread searches its own row, one barrier per pivot; both measured slower)
_OSD_MODES = {"default": {}, "lds": {"QLDPC_OSD_RR": "0"}, "hbm": {"QLDPC_OSD_RR": "0", "QLDPC_OSD_LDS": "0"},
              "pnl1": {"QLDPC_OSD_PNL": "1"}, "pnl2": {"QLDPC_OSD_PNL": "2"}, "blk": {"QLDPC_OSD_PNL": "3"},
              "blk2": {"QLDPC_OSD_PNL": "3", "QLDPC_OSD_RPT": "2"},
              # the lagged one-barrier loop (pivot word applied at once, the rest one step later)
              "lag": {"QLDPC_OSD_PNL": "4"},
              # forward elimination with compaction + blocked back substitution (osd_cs: lean loop)
              "fwd": {"QLDPC_OSD_PNL": "5"},
              # the lean loop with two rows per thread (384-thread workgroups, two per CU)
              "rpt2": {"QLDPC_OSD_RPT": "2"},
              # the opt-in column window (measured slower): its own width (rank + nh
              # + 64 positions), forced to 8 words, its full-width redo exercised on every odd
              # syndrome, and the one-workgroup-per-CU build of the window kernel
              "win": {"QLDPC_OSD_WIN": "1"}, "win8": {"QLDPC_OSD_WIN": "8"},
              "winredo": {"QLDPC_OSD_WIN": "1", "QLDPC_OSD_WIN_REDO": "1"},
              "wpe3": {"QLDPC_OSD_WIN": "1", "QLDPC_OSD_WPE": "3"}}
# the product modes: register rows, and the LDS image / HBM slice that serve graphs past them (the
# switches only force them); the rest are measured-and-not-kept variants compiled into experimental
# builds only (-DQLDPC_EXPERIMENTAL=1, tools/build_variant.py): skipped in the product build


def _set_osd_mode(monkeypatch, mode):
    from qldpc_fault_tolerance_amd import _native

    if mode not in ("default", "lds", "hbm") and not _native.experimental_families():
        pytest.skip(f"OSD mode {mode!r}: experimental builds only")
    for k, v in _OSD_MODES[mode].items():
        monkeypatch.setenv(k, v)


@pytest.mark.parametrize("name,t0,method,order,mode", [
    ("hgp_34_n225", 0, "osd_e", 10, "default"), ("hgp_34_n225", 0, "osd_cs", 8, "default"), ("hgp_34_n225", 0, "osd_0", 0, "default"),
    ("hgp_34_n1600", 0, "osd_e", 10, "default"), ("hgp_34_n1600", 0, "osd_cs", 6, "default"), ("hgp_34_n225", 3, "osd_e", 8, "default"),
    ("hgp_34_n225", 0, "osd_e", 10, "lds"), ("hgp_34_n1600", 0, "osd_e", 10, "lds"), ("hgp_34_n225", 3, "osd_e", 8, "lds"),
    ("hgp_34_n225", 0, "osd_e", 10, "hbm"), ("hgp_34_n1600", 0, "osd_cs", 6, "hbm"), ("hgp_34_n225", 3, "osd_e", 8, "hbm"),
    ("hgp_34_n1600", 0, "osd_e", 10, "pnl1"), ("hgp_34_n225", 3, "osd_e", 8, "pnl1"),
    ("hgp_34_n225", 0, "osd_cs", 8, "pnl2"), ("hgp_34_n1600", 0, "osd_e", 10, "pnl2"), ("hgp_34_n225", 3, "osd_e", 8, "pnl2"),
    ("hgp_34_n225", 0, "osd_e", 10, "blk"), ("hgp_34_n225", 0, "osd_cs", 8, "blk"), ("hgp_34_n1600", 0, "osd_e", 10, "blk"),
    ("hgp_34_n1600", 0, "osd_cs", 6, "blk"), ("hgp_34_n225", 3, "osd_e", 8, "blk"), ("LP_Matg8_L30_Dmin20", 0, "osd_e", 10, "blk"),
    ("hgp_34_n1600", 0, "osd_e", 10, "win"), ("hgp_34_n1600", 0, "osd_e", 10, "winredo"),
    ("hgp_34_n1600", 0, "osd_e", 10, "blk2"),
    ("hgp_34_n1600", 0, "osd_e", 10, "wpe3"), ("hgp_34_n1600", 0, "osd_0", 0, "win"),
    ("LP_Matg8_L30_Dmin20", 0, "osd_e", 10, "win"), ("LP_Matg8_L30_Dmin20", 0, "osd_e", 10, "win8"),
    ("LP_Matg8_L30_Dmin20", 0, "osd_e", 20, "winredo"), ("hgp_34_n225", 3, "osd_e", 8, "winredo"),
    ("hgp_34_n225", 3, "osd_0", 0, "win8"),
    ("hgp_34_n225", 0, "osd_e", 10, "lag"), ("hgp_34_n225", 0, "osd_cs", 8, "lag"), ("hgp_34_n225", 0, "osd_0", 0, "lag"),
    ("hgp_34_n1600", 0, "osd_e", 10, "lag"), ("hgp_34_n1600", 0, "osd_cs", 6, "lag"), ("hgp_34_n225", 3, "osd_e", 8, "lag"),
    ("LP_Matg8_L30_Dmin20", 0, "osd_e", 10, "lag"),
    ("hgp_34_n225", 0, "osd_e", 10, "fwd"), ("hgp_34_n225", 0, "osd_0", 0, "fwd"), ("hgp_34_n1600", 0, "osd_e", 10, "fwd"),
    ("hgp_34_n1600", 0, "osd_0", 0, "fwd"), ("hgp_34_n225", 3, "osd_e", 8, "fwd"), ("LP_Matg8_L30_Dmin20", 0, "osd_e", 10, "fwd"),
    ("LP_Matg8_L30_Dmin20", 0, "osd_e", 20, "fwd"), ("hgp_34_n1600", 0, "osd_cs", 6, "fwd"),
    ("hgp_34_n1600", 0, "osd_e", 10, "rpt2"), ("hgp_34_n1600", 0, "osd_cs", 6, "rpt2"), ("hgp_34_n1600", 0, "osd_0", 0, "rpt2")])
def test_gpu_osd_matches_host_osd(gpu, monkeypatch, name, t0, method, order, mode):
    """GPU OSD kernel == native host OSD stage (itself pinned to the oracle in
    tests/test_osd_cpu.py) on GPU soft-BP posteriors, incl. a rank-deficient space-time graph
    (t0 = 3 repetitions), in each elimination mode of the kernel (every reference code takes the
    register rows by default; the LDS image and the HBM slice serve wider graphs)."""
    from qldpc_fault_tolerance_amd.engine import DeviceBP, DeviceOSD, HostOSD

    _set_osd_mode(monkeypatch, mode)

    code = codes.get_code(name)
    H = code.hz if t0 == 0 else codes.space_time_csr(code.hz, t0).to_dense().astype(np.uint8)
    n = H.shape[1]
    p = 0.05 if t0 else (0.09 if n < 1000 else 0.06)
    synd, _ = _sample(H, p, 192, seed=len(method) + order)
    bp = DeviceBP(H, p, max_iter=max(1, int(code.N / 10)), ms_scaling_factor=0.625, precision=64, soft=True)
    osd = DeviceOSD(bp.graph, np.full(n, p), method, order)
    geo = osd.geometry()
    if mode == "win8":
        assert geo["window_words"] == 8
    elif mode not in ("win", "winredo", "wpe3") or method == "osd_cs" or n < 500:
        assert geo["window_words"] == 0
    else:  # rank + nh + 64 positions fit fewer words than the rows
        assert 0 < geo["window_words"] < geo["row_words"], geo
    ow, o0, corr, iters, conv, post = osd.bposd_batch(bp, synd)
    assert (~conv).sum() > 0
    h0, hw = HostOSD(H, np.full(n, p), method, order).decode_batch(synd, post, conv, corr)
    assert np.array_equal(o0, h0)
    assert np.array_equal(ow, hw)
    assert np.array_equal((H.astype(np.int64) @ ow.T.astype(np.int64) % 2).T, synd)
    assert DeviceOSD.supported(n, p, method, order) and DeviceOSD.supported(n, np.linspace(.01, .1, n), method, 1)


@pytest.mark.parametrize("name,method,order,mode", [
    ("hgp_34_n225", "osd_e", 10, "default"), ("hgp_34_n225", "osd_cs", 8, "default"), ("hgp_34_n225", "osd_0", 0, "default"),
    ("hgp_34_n1600", "osd_e", 10, "default"), ("hgp_34_n225", "osd_e", 10, "lds"), ("hgp_34_n225", "osd_e", 8, "hbm"),
    ("circuit_h2_all3c", "osd_e", 10, "default"), ("circuit_h2_demo", "osd_e", 10, "default"),
    ("hgp_34_n1600", "osd_e", 10, "blk"), ("circuit_h1_all3r", "osd_cs", 6, "blk"),
    ("circuit_h1_all3r", "osd_cs", 6, "default"), ("hgp_34_n1600", "osd_e", 10, "winredo"),
    ("hgp_34_n1600", "osd_e", 10, "win"), ("hgp_34_n1600", "osd_e", 10, "lag"),
    ("circuit_h2_demo", "osd_e", 10, "lag"), ("circuit_h1_all3r", "osd_cs", 6, "lag"),
    ("hgp_34_n1600", "osd_e", 10, "fwd"), ("circuit_h2_demo", "osd_e", 10, "fwd"), ("circuit_h2_all3c", "osd_e", 10, "fwd"),
    ("hgp_34_n1600", "osd_e", 10, "rpt2")])
def test_gpu_osd_nonuniform_priors_matches_oracle(gpu, oracle, monkeypatch, name, method, order, mode):
    """GPU OSD with NON-uniform channel_probs (the circuit-level final round
    ST_BPOSD_Decoder_Circuit(h2, channel_ps2, ...), src/Decoders_SpaceTime.py:277-292): candidates
    weighed by sum log(1/p_j) in ascending column order (osd.hip step 6') == the oracle's literal OSD
    (oracle.osd_decode: Neal LU, per-candidate solve, soft weight summed in index order) and the
    native host stage, per syndrome.  Graphs: codes with drawn priors, and the reference-generated
    circuit hypergraphs with their DEM priors (tests/golden/reference_circuit.npz)."""
    from qldpc_fault_tolerance_amd.engine import DeviceBP, DeviceOSD, HostOSD

    _set_osd_mode(monkeypatch, mode)
    if name.startswith("circuit_"):
        import os

        _, h, tag = name.split("_")
        z = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_circuit.npz"))
        H = z[f"{tag}_exact_{h}"].astype(np.uint8)
        probs = z[f"{tag}_exact_channel_ps{h[1]}"].astype(np.float64)
        # circuit-level rates are tiny; scale the error draw up so BP leaves non-converged syndromes
        rng = np.random.default_rng(order + len(name))
        e = (rng.random((256, H.shape[1])) < np.minimum(0.25, 40 * probs)).astype(np.uint8)
        synd = (e.astype(np.int64) @ H.T.astype(np.int64) % 2).astype(np.uint8)
        mi = 2
    else:
        code = codes.get_code(name)
        H = code.hz
        n = H.shape[1]
        rng = np.random.default_rng(11 + order)
        probs = rng.uniform(0.02, 0.12, n)
        probs[::7] = probs[3]  # some equal priors: tied soft weights occur
        synd, _ = _sample(H, 0.08 if n < 1000 else 0.055, 192, seed=order + 5)
        mi = int(n / 10)
    n = H.shape[1]
    assert DeviceOSD.supported(n, probs, method, order)
    bp = DeviceBP(H, probs, max_iter=mi, ms_scaling_factor=0.625, precision=64, soft=True)
    osd = DeviceOSD(bp.graph, probs, method, order)
    ow, o0, corr, iters, conv, post = osd.bposd_batch(bp, synd)
    assert (~conv).sum() > 0
    h0, hw = HostOSD(H, probs, method, order).decode_batch(synd, post, conv, corr)
    assert np.array_equal(o0, h0) and np.array_equal(ow, hw)
    idx = np.flatnonzero(~conv)[:48]
    if n < 1000:  # the literal numpy restatement
        for b in idx:
            r0, rw = oracle.osd_decode(H, probs, synd[b], post[b], method, order)
            assert np.array_equal(ow[b], rw) and np.array_equal(o0[b], r0), b
    else:  # its C restatement (the same algorithm step for step), fast enough for n1600
        r0, rw = oracle.osd_decode_batch(H, probs, synd[idx], post[idx], method, order)
        assert np.array_equal(ow[idx], rw) and np.array_equal(o0[idx], r0)
    assert np.array_equal((H.astype(np.int64) @ ow.T.astype(np.int64) % 2).T, synd)


def test_bposd_decoder_host_and_gpu_osd_agree(gpu):
    from qldpc_fault_tolerance_amd.decoders import BPOSD_Decoder

    code = codes.get_code("hgp_34_n225")
    synd, _ = _sample(code.hx, 0.1, 128, seed=3)
    a = BPOSD_Decoder(code.hx, 0.1 * np.ones(code.N), 22, "minimum_sum", 0.625, "osd_e", 10)
    b = BPOSD_Decoder(code.hx, 0.1 * np.ones(code.N), 22, "minimum_sum", 0.625, "osd_e", 10, use_gpu_osd=False)
    assert a.gpu_osd is not None and b.gpu_osd is None
    assert np.array_equal(a.decode_batch(synd), b.decode_batch(synd))
    pr = np.random.default_rng(5).uniform(0.03, 0.15, code.N)  # non-uniform priors: the GPU OSD too
    a = BPOSD_Decoder(code.hx, pr, 22, "minimum_sum", 0.625, "osd_e", 10)
    b = BPOSD_Decoder(code.hx, pr, 22, "minimum_sum", 0.625, "osd_e", 10, use_gpu_osd=False)
    assert a.gpu_osd is not None and b.gpu_osd is None
    assert np.array_equal(a.decode_batch(synd), b.decode_batch(synd))


def test_phenl_space_time_with_bposd_final_round(gpu, oracle):
    """CodeSimulator_Phenon_SpaceTime with decoder2 = BPOSD_Decoder (the notebooks'
    final-round decoder): the staged GPU pipeline runs soft BP + GPU OSD on the
    perfect round.  Same seed as with a BP final round: identical detector
    traces (noise and ST decodes do not depend on decoder2); per sample the BP+OSD
    verdicts equal the oracle's (BP then the C OSD restatement on the final round), and
    fail only where the BP verdicts fail, with strictly fewer sector failures here."""
    from qldpc_fault_tolerance_amd.decoders import BPOSD_Decoder_Class, ST_BP_Decoder_Class
    from qldpc_fault_tolerance_amd.engine import DeviceBP, DeviceOSD, DevicePhenl

    code = codes.get_code("hgp_34_n225")
    p, rep, rounds, S = 0.01, 3, 3, 3000
    n = code.N
    mi = int(n / 10)

    def st(H, m):
        return DeviceBP(codes.space_time_csr(H, rep), np.hstack([p * np.ones(n), p * np.ones(m)] * rep),
                        max_iter=mi, precision=64)

    def run(osd):
        d2x = DeviceBP(code.hz, p, max_iter=mi, precision=64, soft=osd)
        d2z = DeviceBP(code.hx, p, max_iter=mi, precision=64, soft=osd)
        ph = DevicePhenl(code, st(code.hz, code.hz.shape[0]), st(code.hx, code.hx.shape[0]), d2x, d2z,
                         num_rep=rep)
        if osd:
            ph.set_final_osd(DeviceOSD(d2x.graph, p * np.ones(n), "osd_e", 10),
                             DeviceOSD(d2z.graph, p * np.ones(n), "osd_e", 10))
        return ph.run(p / 2, p / 2, p / 2, p, 4242, 0, S, rounds, "Total", per_shot=True)

    bp, bo = run(False), run(True)
    assert np.array_equal(bp.trace, bo.trace)
    # per-sample parity with the oracle's BP + OSD restatement of the final round
    ref = oracle.phenl_run(code, p / 2, p / 2, p / 2, p, 4242, 0, S, rounds, rep, "Total", p_data=p, p_synd=p,
                           per_shot=True, osd_method="osd_e", osd_order=10)
    assert np.array_equal(bo.trace, ref["trace"]) and np.array_equal(bo.fail, ref["fail"])
    assert bo.failures == ref["failures"] and bo.sector_fail == ref["sector_fail"]
    assert not np.any((bo.fail != 0) & (bp.fail == 0))
    assert bo.failures <= bp.failures
    assert sum(bo.sector_fail) < sum(bp.sector_fail)
    # the simulator routes BPOSD decoder2 objects onto that pipeline
    from qldpc_fault_tolerance_amd.simulators import CodeSimulator_Phenon_SpaceTime

    d1 = ST_BP_Decoder_Class(10, "minimum_sum", 0.625)
    d2 = BPOSD_Decoder_Class(10, "minimum_sum", 0.625, "osd_e", 10)
    ps = {"p_data": p, "p_syndrome": p, "num_rep": rep}
    sim = CodeSimulator_Phenon_SpaceTime(code, d1.GetDecoder({**ps, "h": code.hz}), d1.GetDecoder({**ps, "h": code.hx}),
                                         d2.GetDecoder({"h": code.hz, "p_data": p}),
                                         d2.GetDecoder({"h": code.hx, "p_data": p}), pauli_error_probs=[p / 2] * 3,
                                         q=p, eval_logical_type="Total", num_rep=rep, seed=4242)
    assert sim._engine_parts() is not None and all(o is not None for o in sim._final_osd())
    res = sim.fused_counts(rounds, 512)
    assert res.shots == 512


def test_phen_single_shot_bpdecoder_bposd_notebook_config(gpu, oracle):
    """The Threshold notebook's CodeFamilyPhenlThreshold pair: decoder1 = BPDecoder on [h | I],
    decoder2 = BPOSD_Decoder osd_e(10).  CodeSimulator_Phenon routes it onto the fused
    pipeline (qldpc_phenl_set_final_osd): the detector trace equals the oracle's (num_rep = 1) and
    the BP-final-round run's, the per-sample BP+OSD verdicts equal the oracle's BP + OSD
    restatement, and BP+OSD fails only where BP fails."""
    from qldpc_fault_tolerance_amd.decoders import BP_Decoder_Class, BPOSD_Decoder_Class
    from qldpc_fault_tolerance_amd.simulators import CodeSimulator_Phenon

    code = codes.get_code("hgp_34_n225")
    p, rounds, S = 0.02, 3, 1500
    ext = lambda h: np.hstack([h, np.identity(h.shape[0])])  # noqa: E731
    b1 = BP_Decoder_Class(10, "minimum_sum", 0.625)
    d1 = {"p_data": p, "p_syndrome": p}

    def sim(dec2_cls):
        return CodeSimulator_Phenon(code, b1.GetDecoder({**d1, "h": ext(code.hz)}), b1.GetDecoder({**d1, "h": ext(code.hx)}),
                                    dec2_cls.GetDecoder({"h": code.hz, "p_data": p}),
                                    dec2_cls.GetDecoder({"h": code.hx, "p_data": p}), pauli_error_probs=[p / 2] * 3,
                                    q=p, eval_logical_type="Total", seed=31)

    s_osd = sim(BPOSD_Decoder_Class(10, "minimum_sum", 0.625, "osd_e", 10))
    assert s_osd._engine_parts() is not None and all(o is not None for o in s_osd._final_osd())
    s_bp = sim(b1)
    from qldpc_fault_tolerance_amd.engine import DevicePhenl

    runs = []
    for s in (s_bp, s_osd):
        ph = DevicePhenl(code, *s._engine_parts(), num_rep=1)
        ox, oz = s._final_osd()
        if ox is not None:
            ph.set_final_osd(ox, oz)
        runs.append(ph.run(p / 2, p / 2, p / 2, p, 31, 0, S, rounds, "Total", per_shot=True))
    bp, bo = runs
    ref = oracle.phenl_run(code, p / 2, p / 2, p / 2, p, 31, 0, S, rounds, 1, "Total", p_data=p, p_synd=p,
                           per_shot=True)
    assert np.array_equal(bp.trace, ref["trace"]) and np.array_equal(bp.fail, ref["fail"])
    assert np.array_equal(bo.trace, bp.trace)
    ref_osd = oracle.phenl_run(code, p / 2, p / 2, p / 2, p, 31, 0, S, rounds, 1, "Total", p_data=p, p_synd=p,
                               per_shot=True, osd_method="osd_e", osd_order=10)
    assert np.array_equal(bo.fail, ref_osd["fail"]) and bo.sector_fail == ref_osd["sector_fail"]
    assert not np.any((bo.fail != 0) & (bp.fail == 0))
    assert bo.failures <= bp.failures
    # the drop-in's fused path returns the same count as the device run of the same stream
    assert s_osd.fused_counts(rounds, S).failures == bo.failures


def test_final_osd_graph_mismatch_is_rejected(gpu):
    """qldpc_phenl_set_final_osd refuses an OSD handle built on another graph."""
    from qldpc_fault_tolerance_amd import _native
    from qldpc_fault_tolerance_amd.engine import DeviceBP, DeviceOSD, DevicePhenl

    code = codes.get_code("hgp_34_n225")
    p, n = 0.02, code.N
    st = [DeviceBP(codes.space_time_csr(h, 1), np.full(n + h.shape[0], p), max_iter=22) for h in (code.hz, code.hx)]
    d2x = DeviceBP(code.hz, p, max_iter=22, soft=True)
    d2z = DeviceBP(code.hx, p, max_iter=22, soft=True)
    ph = DevicePhenl(code, st[0], st[1], d2x, d2z, num_rep=1)
    ox, oz = DeviceOSD(d2x.graph, np.full(n, p), "osd_e", 4), DeviceOSD(d2z.graph, np.full(n, p), "osd_e", 4)
    with pytest.raises(_native.QldpcError, match="different graph"):
        ph.set_final_osd(oz, ox)  # swapped sectors
    ph.set_final_osd(ox, oz)


def _oracle_sector_fails(oracle, code, err, p, mi, order, method="osd_e"):
    """Per shot and sector: the reference's BPOSD verdict on the engine's sampled errors —
    oracle BP (soft), then the C OSD restatement where BP did not converge, then the
    _single_run failure check (src/Simulators.py:135-160)."""
    from qldpc_fault_tolerance_amd.simulators import gf2_rows

    out = np.zeros((err.shape[0], 2), dtype=bool)
    for q, H, L, k in ((0, code.hz, code.lz, "hz"), (1, code.hx, code.lx, "hx")):
        e = ((err >> q) & 1).astype(np.uint8)
        synd = gf2_rows(code.csr(k), e)
        oc, _, ov, op = oracle.bp_decode_batch_soft(H, p, mi, 0.625, synd, 64)
        x = oc.copy()
        nc = np.flatnonzero(~ov)
        if nc.size:
            x[nc] = oracle.osd_decode_batch(H, p * np.ones(code.N), synd[nc], op[nc], method, order)[1]
        r = (e ^ x).astype(np.uint8)
        out[:, q] = gf2_rows(code.csr(k), r).any(1) | gf2_rows(code.csr("lz" if q == 0 else "lx"), r).any(1)
    return out


def test_bposd_shot_loop_n1600_osd_e10_matches_oracle_per_shot(gpu, oracle):
    """The fused BP+OSD shot loop (qldpc_mc_set_osd) at the headline code with the notebooks'
    OSD-E(10): per shot and sector the verdict equals the oracle's BP + OSD restatement on the
    same Philox errors (n1600 OSD-E(10) parity through the fused loop)."""
    from qldpc_fault_tolerance_amd.decoders import BPOSD_Decoder_Class
    from qldpc_fault_tolerance_amd.simulators import CodeSimulator_DataError

    code = codes.get_code("hgp_34_n1600")
    p, S = 0.05, 384
    cls = BPOSD_Decoder_Class(10, "minimum_sum", 0.625, "osd_e", 10)
    dx, dz = cls.GetDecoder({"h": code.hz, "p_data": p}), cls.GetDecoder({"h": code.hx, "p_data": p})
    sim = CodeSimulator_DataError(code, dx, dz, [p / 2] * 3, "Total", seed=1600)
    fails, shots, osd_n = sim.bposd_counts(S, keep_shots=True)
    assert sim._bposd_dev, "the device-resident loop must serve the headline code"
    assert shots == S and osd_n >= 40
    err, sf = sim.last_shots
    ref = _oracle_sector_fails(oracle, code, err, p, int(code.N / 10), 10)
    assert np.array_equal(sf, ref)
    assert fails == int((ref[:, 0] | ref[:, 1]).sum())


@pytest.mark.parametrize("env", [{"QLDPC_MC_STAGED": "1"}, {"QLDPC_ENGINE": "2"}])
def test_bposd_shot_loop_off_engine3_takes_host_path(gpu, oracle, monkeypatch, env):
    """with the fused engine-3 MC unavailable (staged pipeline, a forced engine)
    bposd_counts keeps the host-assisted loop instead of raising, with the oracle's verdicts."""
    from qldpc_fault_tolerance_amd.decoders import BPOSD_Decoder_Class
    from qldpc_fault_tolerance_amd.simulators import CodeSimulator_DataError

    for k, v in env.items():
        monkeypatch.setenv(k, v)
    code = codes.get_code("hgp_34_n225")
    p, order, S = 0.08, 4, 160
    cls = BPOSD_Decoder_Class(10, "minimum_sum", 0.625, "osd_e", order)
    dx, dz = cls.GetDecoder({"h": code.hz, "p_data": p}), cls.GetDecoder({"h": code.hx, "p_data": p})
    sim = CodeSimulator_DataError(code, dx, dz, [p / 2] * 3, "Total", seed=77)
    fails, shots, osd_n = sim.bposd_counts(S, batch=64, keep_shots=True)
    assert not sim._bposd_dev  # routed to the host-assisted loop
    assert shots == S and osd_n > 0
    err, sf = sim.last_shots
    ref = _oracle_sector_fails(oracle, code, err, p, int(code.N / 10), order)
    assert np.array_equal(sf, ref)
    assert fails == int((ref[:, 0] | ref[:, 1]).sum())


def test_bposd_capture_budget_splits_launch_identically(gpu, monkeypatch):
    """capture slots are bounded (QLDPC_OSD_CAPTURE_MB); a launch with more shots
    than slots runs as pieces.  1 MB -> 1024 slots at n225: a 5000-shot launch in 5 pieces gives
    the same per-shot errors, verdicts and counters as one piece."""
    from qldpc_fault_tolerance_amd.decoders import BPOSD_Decoder_Class
    from qldpc_fault_tolerance_amd.simulators import CodeSimulator_DataError

    code = codes.get_code("hgp_34_n225")
    p, S = 0.09, 5000
    cls = BPOSD_Decoder_Class(10, "minimum_sum", 0.625, "osd_e", 6)

    def run():
        dx, dz = cls.GetDecoder({"h": code.hz, "p_data": p}), cls.GetDecoder({"h": code.hx, "p_data": p})
        sim = CodeSimulator_DataError(code, dx, dz, [p / 2] * 3, "Total", seed=5)
        r = sim.bposd_counts(S, batch=S, keep_shots=True)
        return r, sim.last_shots, sim.last_result

    a, (ea, fa), ra = run()
    monkeypatch.setenv("QLDPC_OSD_CAPTURE_MB", "1")
    b, (eb, fb), rb = run()
    assert a == b and a[2] > 1024  # more candidates than one piece's slots
    assert np.array_equal(ea, eb) and np.array_equal(fa, fb)
    assert ra.sector_fail == rb.sector_fail and ra.sector_iters == rb.sector_iters
