"""GPU parity of the phenomenological space-time shot loop (qldpc_phenl_*).

Reference: CodeSimulator_Phenon_SpaceTime (src/Simulators_SpaceTime.py:382-548)
with ST_BP_Decoder_syndrome (src/Decoders_SpaceTime.py:200-223) as decoder1.
The golden case replays CPython's own random() stream (uniforms recorded by
tests/golden/make_golden.py from the reference harness); the Philox cases
compare against the oracle's restatement (oracle_phenl_run) bit for bit.
"""
import os

import numpy as np
import pytest

from qldpc_fault_tolerance_amd import codes, decoders, simulators
from qldpc_fault_tolerance_amd.engine import DeviceBP, DevicePhenl

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_harness_n225.npz")


def _phenl(code, p_data, p_synd, num_rep, precision, max_iter=None, max_batch=0):
    n = code.N
    mi = int(n / 10) if max_iter is None else max_iter
    hz, hx = code.csr("hz"), code.csr("hx")
    pst_x = np.hstack([p_data * np.ones(n), p_synd * np.ones(hz.m)] * num_rep)
    pst_z = np.hstack([p_data * np.ones(n), p_synd * np.ones(hx.m)] * num_rep)
    st_x = DeviceBP(codes.space_time_csr(code.hz, num_rep), pst_x, max_iter=mi, precision=precision)
    st_z = DeviceBP(codes.space_time_csr(code.hx, num_rep), pst_z, max_iter=mi, precision=precision)
    d2x = DeviceBP(hz, p_data * np.ones(n), max_iter=mi, precision=precision)
    d2z = DeviceBP(hx, p_data * np.ones(n), max_iter=mi, precision=precision)
    return DevicePhenl(code, st_x, st_z, d2x, d2z, num_rep=num_rep, max_batch=max_batch)


def _split_trace(tr, num_rounds, num_rep, m):
    """[S, trace_len] -> (z histories [S*(R-1), rep, m], x histories, final z synd [S, m], final x synd)."""
    S = tr.shape[0]
    R1 = num_rounds - 1
    body = tr[:, :R1 * 2 * num_rep * m].reshape(S, R1, 2, num_rep, m)
    fin = tr[:, R1 * 2 * num_rep * m:].reshape(S, 2, m)
    return (body[:, :, 0].reshape(S * R1, num_rep, m), body[:, :, 1].reshape(S * R1, num_rep, m),
            fin[:, 0], fin[:, 1])


def test_phenl_replays_reference_harness(gpu):
    """External CPython uniforms: detector histories, final syndromes and failures == the reference harness."""
    g = np.load(GOLD)
    code = codes.get_code("hgp_34_n225")
    p = 0.02
    ph = _phenl(code, p, p, 3, precision=64)
    U = g["phenst_u"]
    res = ph.run(p / 2, p / 2, p / 2, p, seed=0, shot_begin=0, shot_count=U.shape[0], num_rounds=3,
                 logical_mode="Total", uniforms=U, per_shot=True)
    hz_, hx_, fz, fx = _split_trace(res.trace, 3, 3, code.hz.shape[0])
    assert np.array_equal(hz_, g["phenst_d1z_hist"])
    assert np.array_equal(hx_, g["phenst_d1x_hist"])
    assert np.array_equal(fz, g["phenst_d2z_synd"])
    assert np.array_equal(fx, g["phenst_d2x_synd"])
    assert np.array_equal((res.fail != 0).astype(np.uint8), g["phenst_fail"])
    assert res.failures == int(g["phenst_fail"].sum()) and res.shots == U.shape[0]


@pytest.mark.parametrize("precision", [64, 32])
@pytest.mark.parametrize("mode", ["Total", "X", "Z"])
def test_phenl_philox_matches_oracle(gpu, oracle, precision, mode):
    code = codes.get_code("hgp_34_n225")
    p = 0.03
    S, R, rep = 333, 4, 3  # 333: a ragged last sample word
    ph = _phenl(code, p, p, rep, precision)
    res = ph.run(p / 2, p / 2, p / 2, p, seed=77, shot_begin=1000, shot_count=S, num_rounds=R, logical_mode=mode,
                 per_shot=True)
    ref = oracle.phenl_run(code, p / 2, p / 2, p / 2, p, 77, 1000, S, R, rep, mode, p_data=p, p_synd=p,
                           precision=precision, per_shot=True)
    assert np.array_equal(res.trace, ref["trace"])
    assert np.array_equal(res.fail, ref["fail"])
    assert res.failures == ref["failures"] and res.shots == S
    assert res.sector_decodes == ref["sector_decodes"]
    assert res.sector_iters == ref["sector_iters"]
    assert res.sector_nonconv == ref["sector_nonconv"]
    assert res.sector_fail == ref["sector_fail"]


def test_phenl_chunking_and_sharding_invariance(gpu):
    """Counters do not depend on max_batch chunking or on how the sample range is split (per-sample RNG keys)."""
    code = codes.get_code("hgp_34_n225")
    p = 0.04
    a = _phenl(code, p, p, 2, precision=32).run(p / 2, p / 2, p / 2, p, 5, 0, 1000, 3, per_shot=True)
    b = _phenl(code, p, p, 2, precision=32, max_batch=192)
    b1 = b.run(p / 2, p / 2, p / 2, p, 5, 0, 601, 3, per_shot=True)
    b2 = b.run(p / 2, p / 2, p / 2, p, 5, 601, 399, 3, per_shot=True)
    assert np.array_equal(a.fail, np.concatenate([b1.fail, b2.fail]))
    assert np.array_equal(a.trace, np.concatenate([b1.trace, b2.trace]))
    assert a.failures == b1.failures + b2.failures
    assert a.sector_iters == [x + y for x, y in zip(b1.sector_iters, b2.sector_iters)]


def test_phenl_n1225_space_time_graph(gpu, oracle):
    """Config 5 graph (hgp_34_n1225_q3 stand-in, num_rep=3: ST graph 1764 x 5439) against the oracle, fp32."""
    code = codes.get_code("hgp_34_n1225_q3")
    p = 0.01
    ph = _phenl(code, p, p, 3, precision=32)
    g = ph.decoders[0].geometry()
    # register engine, tail layout with byte F words: two 512-thread decodes per CU (engine id 21013),
    # the 1764 degree-2 measurement variables in 3 compile-time 2-edge slots (+ 100000 * D2K)
    assert (g["engine"], g["kernel_id"], g["threads"], g["vars_per_thread"]) == (3, 321013, 512, 11), g
    assert g["blocks_per_cu"] == 2 and 2 * g["lds_bytes"] <= 160 * 1024, g
    S, R = 96, 3
    res = ph.run(p / 2, p / 2, p / 2, p, 11, 0, S, R, per_shot=True)
    ref = oracle.phenl_run(code, p / 2, p / 2, p / 2, p, 11, 0, S, R, 3, "Total", p_data=p, p_synd=p,
                           precision=32, per_shot=True)
    assert np.array_equal(res.trace, ref["trace"])
    assert np.array_equal(res.fail, ref["fail"])
    assert res.sector_iters == ref["sector_iters"]


def test_phenl_simulator_dropin(gpu, oracle):
    """CodeSimulator_Phenon_SpaceTime.WordErrorRate (fused path) == the per-cycle formula on the oracle's count."""
    code = codes.get_code("hgp_34_n225")
    eval_p = 0.02
    c1 = decoders.ST_BP_Decoder_Class(max_iter_ratio=10, bp_method="minimum_sum", ms_scaling_factor=0.625)
    c2 = decoders.BP_Decoder_Class(max_iter_ratio=10, bp_method="minimum_sum", ms_scaling_factor=0.625)
    d1x = c1.GetDecoder({"h": code.hz, "p_data": eval_p, "p_syndrome": eval_p, "num_rep": 3})
    d1z = c1.GetDecoder({"h": code.hx, "p_data": eval_p, "p_syndrome": eval_p, "num_rep": 3})
    d2x = c2.GetDecoder({"h": code.hz, "p_data": eval_p})
    d2z = c2.GetDecoder({"h": code.hx, "p_data": eval_p})
    pp = eval_p / 2
    sim = simulators.CodeSimulator_Phenon_SpaceTime(code=code, decoder1_x=d1x, decoder1_z=d1z, decoder2_x=d2x,
                                                    decoder2_z=d2z, pauli_error_probs=[pp] * 3, q=eval_p,
                                                    eval_logical_type="Total", num_rep=3, seed=99)
    wer, none = sim.WordErrorRate(num_cycles=7, num_samples=500)  # num_rounds = 3
    ref = oracle.phenl_run(code, pp, pp, pp, eval_p, 99, 0, 500, 3, 3, "Total", p_data=eval_p, p_synd=eval_p)
    assert none is None
    assert wer == simulators.word_error_rate_per_cycle(ref["failures"], 500, code.K, 7)


# ------------------------------------------------ single-shot phenomenological (CodeSimulator_Phenon, num_rep = 1)
PHEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_harness_phen_n225.npz")


def _phen_dropin(code, p, seed=None, precision=64):
    cls = decoders.BP_Decoder_Class(max_iter_ratio=10, bp_method="minimum_sum", ms_scaling_factor=0.625,
                                    precision=precision)
    ext = lambda h: np.hstack([h, np.identity(h.shape[0])])  # noqa: E731
    d1x = cls.GetDecoder({"h": ext(code.hz), "p_data": p, "p_syndrome": p})
    d1z = cls.GetDecoder({"h": ext(code.hx), "p_data": p, "p_syndrome": p})
    d2x = cls.GetDecoder({"h": code.hz, "p_data": p})
    d2z = cls.GetDecoder({"h": code.hx, "p_data": p})
    return simulators.CodeSimulator_Phenon(code=code, decoder1_x=d1x, decoder1_z=d1z, decoder2_x=d2x,
                                           decoder2_z=d2z, pauli_error_probs=[p / 2] * 3, q=p,
                                           eval_logical_type="Total", seed=seed)


def test_phen_single_shot_replays_reference_harness(gpu):
    """CodeSimulator_Phenon on the GPU (DevicePhenl, num_rep=1) replays the reference harness bit for bit."""
    g = np.load(PHEN)
    code = codes.get_code("hgp_34_n225")
    p, m = 0.02, code.hz.shape[0]
    sim = _phen_dropin(code, p)
    from qldpc_fault_tolerance_amd.engine import DevicePhenl

    ph = DevicePhenl(code, *sim._engine_parts(), num_rep=1)
    res = ph.run(p / 2, p / 2, p / 2, p, 0, 0, 16, 3, "Total", uniforms=g["phen_u"], per_shot=True)
    body = res.trace[:, :4 * m].reshape(16, 2, 2, m)
    assert np.array_equal(body[:, :, 0].reshape(32, m), g["phen_d1z_synd"])
    assert np.array_equal(body[:, :, 1].reshape(32, m), g["phen_d1x_synd"])
    assert np.array_equal(res.trace[:, 4 * m:5 * m], g["phen_d2z_synd"])
    assert np.array_equal(res.trace[:, 5 * m:], g["phen_d2x_synd"])
    assert np.array_equal((res.fail != 0).astype(np.uint8), g["phen_fail"])


def test_phen_single_shot_dropin_matches_oracle(gpu, oracle):
    code = codes.get_code("hgp_34_n225")
    p = 0.02
    sim = _phen_dropin(code, p, seed=2024)
    wer, none = sim.WordErrorRate(5, 700)
    ref = oracle.phenl_run(code, p / 2, p / 2, p / 2, p, 2024, 0, 700, 5, 1, "Total", p_data=p, p_synd=p)
    assert none is None
    assert wer == simulators.word_error_rate_phenl(ref["failures"], 700, code.K, 5)
    assert sim.last_result.sector_iters == ref["sector_iters"]


@pytest.mark.parametrize("dec2", ["bp", "bposd"])
def test_phen_single_shot_firstmin_decoder1_fused_matches_oracle(gpu, oracle, dec2):
    """CodeSimulator_Phenon with FirstMinBPDecoder decoder1 (the Single-Shot notebook's configuration:
    p_data = p_synd = 2p/3 on [h | I], max_iter = N/10) runs fused (qldpc_phenl_set_round_firstmin) and
    equals the oracle's pipeline with the reference's first-min loop per noisy round: failures, per-sector
    failures, accepted steps and the final round's iterations; decoder2 BP or BPOSD osd_e(10)."""
    code = codes.get_code("hgp_34_n225")
    p = 0.03
    pd = 2 * p / 3
    ext = lambda h: np.hstack([h, np.identity(h.shape[0])])  # noqa: E731
    mi = int(code.N / 10)
    d1x = decoders.FirstMinBPDecoder(ext(code.hz), np.hstack([pd * np.ones(code.N), pd * np.ones(code.hz.shape[0])]),
                                     mi, "minimum_sum", 0.625)
    d1z = decoders.FirstMinBPDecoder(ext(code.hx), np.hstack([pd * np.ones(code.N), pd * np.ones(code.hx.shape[0])]),
                                     mi, "minimum_sum", 0.625)
    pp = 2 * p / 3  # decoder2 channel: (p/3 + p/3)
    if dec2 == "bposd":
        d2x = decoders.BPOSD_Decoder(code.hz, pp * np.ones(code.N), mi, "minimum_sum", 0.625, "osd_e", 10)
        d2z = decoders.BPOSD_Decoder(code.hx, pp * np.ones(code.N), mi, "minimum_sum", 0.625, "osd_e", 10)
    else:
        d2x = decoders.BPDecoder(code.hz, pp * np.ones(code.N), mi, "minimum_sum", 0.625)
        d2z = decoders.BPDecoder(code.hx, pp * np.ones(code.N), mi, "minimum_sum", 0.625)
    sim = simulators.CodeSimulator_Phenon(code=code, decoder1_x=d1x, decoder1_z=d1z, decoder2_x=d2x, decoder2_z=d2z,
                                          pauli_error_probs=[p / 3] * 3, q=pd, eval_logical_type="Total", seed=77)
    assert sim._engine_parts() is not None and sim._firstmin1() is not None
    wer, _ = sim.WordErrorRate(5, 600)
    ref = oracle.phenl_run(code, p / 3, p / 3, p / 3, pd, 77, 0, 600, 5, 1, "Total", p_data=pd, p_synd=pd,
                           max_iter_2=mi, firstmin_max_iter=mi, osd_method="osd_e" if dec2 == "bposd" else None)
    res = sim.last_result
    assert res.failures == ref["failures"]
    assert list(res.sector_fail) == list(ref["sector_fail"])
    assert list(res.sector_iters) == list(ref["sector_iters"])
    assert list(res.sector_nonconv) == list(ref["sector_nonconv"])
    assert wer == simulators.word_error_rate_phenl(ref["failures"], 600, code.K, 5)


def test_firstmin_decoder_matches_reference_fixture(gpu):
    """FirstMinBPDecoder (src/Decoders.py:49-74) over the engine == the reference class on the oracle BP."""
    g = np.load(PHEN)
    code = codes.get_code("hgp_34_n225")
    p = 0.02
    hz_ext = np.hstack([code.hz, np.identity(code.hz.shape[0])])
    fm = decoders.FirstMinBPDecoder(hz_ext, np.hstack([p * np.ones(code.N), p * np.ones(code.hz.shape[0])]), 20,
                                    "minimum_sum", 0.625)
    out = fm.decode_batch(g["firstmin_synd"])
    assert np.array_equal(out.astype(np.uint8), g["firstmin_corr"])
    assert np.array_equal(fm.decode(g["firstmin_synd"][3]).astype(np.uint8), g["firstmin_corr"][3])


@pytest.mark.parametrize("kernel", ["wave", "wg"])
@pytest.mark.parametrize("precision,alpha", [(64, 0.625), (32, 0.625), (64, 0.0), (64, 0.9)])
def test_firstmin_device_loop_matches_reference_algorithm(gpu, oracle, monkeypatch, precision, alpha, kernel):
    """The device-resident first-min loop (qldpc_firstmin_*, one kernel) == the reference's
    FirstMinBPDecoder.decode loop (src/Decoders.py:60-74) run over the oracle's one-iteration BP,
    per syndrome (corrections and accepted steps), with non-uniform priors on [h | I], including
    the zero syndrome (every step accepted with an empty correction) and ldpc's alpha = 0 schedule."""
    code = codes.get_code("hgp_34_n225")
    hz_ext = np.hstack([code.hz, np.identity(code.hz.shape[0])]).astype(np.uint8)
    n = hz_ext.shape[1]
    rng = np.random.default_rng(7 + precision + int(alpha * 10))
    probs = rng.uniform(0.005, 0.06, n)
    probs[::5] = probs[2]  # tied priors: equal minima
    e = (rng.random((80, n)) < 0.035).astype(np.uint8)
    synd = (e.astype(np.int64) @ hz_ext.T.astype(np.int64) % 2).astype(np.uint8)
    synd[0] = 0
    mi = 12
    if kernel == "wg":  # one workgroup per syndrome instead of one wave
        monkeypatch.setenv("QLDPC_FM_WAVE", "0")
    fm = decoders.FirstMinBPDecoder(hz_ext, probs, mi, "minimum_sum", alpha, precision=precision)
    out = fm.decode_batch(synd)
    H = hz_ext.astype(np.int64)

    def bp1(s):
        return oracle.bp_decode_batch(hz_ext, probs, 1, "minimum_sum", alpha, s[None].astype(np.uint8),
                                      precision)[0][0].astype(np.int64)

    for b in range(synd.shape[0]):
        corr, cur, k = np.zeros(n, dtype=np.int64), synd[b].astype(np.int64), 0
        nc = bp1(cur)
        ns = (H @ nc + cur) % 2
        while ns.sum() <= cur.sum() and k < mi:
            cur, corr, k = ns, (corr + nc) % 2, k + 1
            nc = bp1(cur)
            ns = (H @ nc + cur) % 2
        assert np.array_equal(out[b], corr), b
        assert fm.steps_batch[b] == k, b
    assert fm.steps_batch[0] == mi and not out[0].any()


@pytest.mark.parametrize("p", [0.01, 0.06])
def test_st_fp32_byte_f_family_decode_matches_oracle(gpu, oracle, p):
    """The fp32 space-time decoder of config 5 on the byte-F family (512 threads x 11 variables,
    2 decodes per CU) against the oracle's float32 restatement and the 1024-thread family
    (QLDPC_E3_FB=0), on syndromes of i.i.d. errors (p = 0.06: every decode runs to max_iter)."""
    import os

    from qldpc_fault_tolerance_amd.engine import DeviceBP

    code = codes.get_code("hgp_34_n1225_q3")
    H = codes.space_time_csr(code.hz, 3)
    n, m = H.n, H.m
    pr = np.full(n, p)
    mi = int(code.N / 10)
    rng = np.random.default_rng(int(p * 1000))
    e = (rng.random((160, n)) < p).astype(np.uint8)
    synd = H.matvec(e).astype(np.uint8)
    dec = DeviceBP(H, pr, max_iter=mi, precision=32)
    assert dec.geometry()["kernel_id"] == 321013
    c, i, v = dec.decode_batch(synd)
    oc, oi, ov = oracle.bp_decode_batch(H, pr, mi, "minimum_sum", 0.625, synd, 32)
    assert np.array_equal(i, oi) and np.array_equal(v, ov) and np.array_equal(c, oc.astype(np.int64))
    # the same family without the degree-2 slots, and the 1024-thread family
    for env, kid in (("QLDPC_D2K", 21013), ("QLDPC_E3_FB", 1013)):
        os.environ[env] = "0"
        try:
            d1 = DeviceBP(H, pr, max_iter=mi, precision=32)
        finally:
            del os.environ[env]
        assert d1.geometry()["kernel_id"] == kid
        c1, i1, v1 = d1.decode_batch(synd)
        assert np.array_equal(c, c1) and np.array_equal(i, i1) and np.array_equal(v, v1), env


@pytest.mark.parametrize("p,alpha", [(0.005, 0.625), (0.06, 0.625), (0.03, 0.0)])
def test_st_fp64_one_word_family_decode_matches_oracle(gpu, oracle, p, alpha):
    """The fp64 space-time decoder of config 5 on the one-word "m2 in slot" tail family (round 6,
    engine id 111313: 1024 threads x 6 variables, own v2c in VGPRs, private dummy slots for the
    measurement / degree-3 variables in wider slots) against the oracle's float64 restatement (the
    reference arithmetic) and the two-word tail family (QLDPC_M2ST=0, engine id 101013), on
    syndromes of i.i.d. errors (p = 0.06: every decode runs to max_iter; alpha 0: ldpc's schedule)."""
    import os

    from qldpc_fault_tolerance_amd.engine import DeviceBP

    code = codes.get_code("hgp_34_n1225_q3")
    H = codes.space_time_csr(code.hz, 3)
    n = H.n
    pr = np.full(n, p)
    mi = int(code.N / 10)
    rng = np.random.default_rng(int(p * 1000) + 17)
    e = (rng.random((192, n)) < p).astype(np.uint8)
    synd = H.matvec(e).astype(np.uint8)
    synd[0] = 0
    dec = DeviceBP(H, pr, max_iter=mi, ms_scaling_factor=alpha, precision=64)
    assert dec.geometry()["kernel_id"] == 111313
    c, i, v = dec.decode_batch(synd)
    oc, oi, ov = oracle.bp_decode_batch(H, pr, mi, "minimum_sum", alpha, synd, 64)
    assert np.array_equal(i, oi) and np.array_equal(v, ov) and np.array_equal(c, oc.astype(np.int64))
    os.environ["QLDPC_M2ST"] = "0"
    try:
        d1 = DeviceBP(H, pr, max_iter=mi, ms_scaling_factor=alpha, precision=64)
    finally:
        del os.environ["QLDPC_M2ST"]
    assert d1.geometry()["kernel_id"] == 101013
    c1, i1, v1 = d1.decode_batch(synd)
    assert np.array_equal(c1, c) and np.array_equal(i1, i) and np.array_equal(v1, v)


def test_st_fp64_nonuniform_priors_keep_two_word_family(gpu, oracle):
    """Non-uniform priors (p_synd != p_data) are outside the one-word family (one prior in SGPRs):
    the two-word tail family decodes them, bit-exact against the oracle."""
    from qldpc_fault_tolerance_amd.engine import DeviceBP

    code = codes.get_code("hgp_34_n1225_q3")
    H = codes.space_time_csr(code.hz, 3)
    pr = np.hstack([0.02 * np.ones(code.N), 0.01 * np.ones(code.hz.shape[0])] * 3)
    rng = np.random.default_rng(5)
    synd = H.matvec((rng.random((64, H.n)) < pr).astype(np.uint8)).astype(np.uint8)
    dec = DeviceBP(H, pr, max_iter=40, precision=64)
    assert dec.geometry()["kernel_id"] == 101013
    c, i, v = dec.decode_batch(synd)
    oc, oi, ov = oracle.bp_decode_batch(H, pr, 40, "minimum_sum", 0.625, synd, 64)
    assert np.array_equal(i, oi) and np.array_equal(v, ov) and np.array_equal(c, oc.astype(np.int64))


def test_firstmin_past_device_envelope_steps_the_engine(gpu, oracle):
    """A minimum_sum FirstMinBPDecoder on a graph past the first-min kernel's LDS envelope (2 (m + n)
    > 64 KiB: QLDPC_ENOTSUP) steps the engine's one-iteration BP from the host instead of raising;
    corrections equal the reference loop (src/Decoders.py:60-74) over the oracle's one-iteration BP.
    max_iter = 2.5 (a float, as N / 10 can be) allows 3 accepted steps, as the reference's raw
    comparison does."""
    rng = np.random.default_rng(11)
    m, n = 12000, 24000
    # column j on rows j, 7 j + 1 and 13 j + 5 (mod m): three distinct rows, every row of degree 6
    j = np.arange(n)
    H = np.zeros((m, n), np.uint8)
    for r in (j % m, (7 * j + 1) % m, (13 * j + 5) % m):
        H[r, j] = 1
    assert (H.sum(0) == 3).all() and (H.sum(1) == 6).all()
    probs = np.full(n, 0.01)
    fm = decoders.FirstMinBPDecoder(H, probs, 2.5, "minimum_sum", 0.625)
    assert fm._fm is None and fm._bp is not None
    e = (rng.random((3, n)) < 0.004).astype(np.uint8)
    synd = (e.astype(np.int64) @ H.T.astype(np.int64) % 2).astype(np.uint8)
    out = fm.decode_batch(synd)
    Hl = H.astype(np.int64)
    for b in range(synd.shape[0]):
        corr, cur, k = np.zeros(n, dtype=np.int64), synd[b].astype(np.int64), 0
        nc = oracle.bp_decode_batch(H, probs, 1, "minimum_sum", 0.625, cur[None].astype(np.uint8), 64)[0][0].astype(np.int64)
        ns = (Hl @ nc + cur) % 2
        while ns.sum() <= cur.sum() and k < 2.5:
            cur, corr, k = ns, (corr + nc) % 2, k + 1
            nc = oracle.bp_decode_batch(H, probs, 1, "minimum_sum", 0.625, cur[None].astype(np.uint8), 64)[0][0].astype(np.int64)
            ns = (Hl @ nc + cur) % 2
        assert np.array_equal(out[b], corr), b
