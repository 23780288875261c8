"""Engine 6 (csrc/bp_hbm.hip): min-sum BP with HBM-resident [edge][lane] messages.

Bit-exact against the oracle (fp64 = ldpc's arithmetic, fp32 = the oracle's float mode) when
forced onto any graph (qldpc_bp_create_hbm; BASELINE config 4 = LP_Matg8_L30_Dmin20), and selected
automatically where no LDS engine holds a decode.  Config 5's fp64 space-time graph at the
drop-in's default precision (ST_BP_Decoder_Class, src/Decoders_SpaceTime.py:200-257) now fits
LDS on engine 3's tail layout (tested here too); forced onto engine 6 it stays bit-exact.
"""
import numpy as np
import pytest

from qldpc_fault_tolerance_amd import codes, decoders

pytestmark = pytest.mark.gpu


def _synd(H, p, B, seed):
    rng = np.random.default_rng(seed)
    e = (rng.random((B, H.shape[1])) < p).astype(np.uint8)
    return (e.astype(np.int64) @ H.T.astype(np.int64) % 2).astype(np.uint8)


@pytest.mark.parametrize("precision", [64, 32])
@pytest.mark.parametrize("name", ["hgp_34_n225", "LP_Matg8_L30_Dmin20", "GenBicycleA3", "hgp_34_n1600"])
def test_hbm_decode_batch_matches_oracle(gpu, oracle, precision, name):
    from qldpc_fault_tolerance_amd.engine import DeviceBP

    code = codes.get_code(name)
    H, n = code.hz, code.N
    mi = int(n / 10)
    for p in (0.02, 0.07):
        synd = _synd(H, p, 333, seed=int(p * 1000) + precision)  # 333: a ragged last 64-lane chunk
        dec = DeviceBP(H, p * np.ones(n), max_iter=mi, precision=precision, hbm=True)
        assert dec.geometry()["engine"] == 6
        corr, iters, conv = dec.decode_batch(synd)
        oc, oi, ov = oracle.bp_decode_batch(H, p, mi, "minimum_sum", 0.625, synd, precision)
        assert np.array_equal(iters, oi), (name, p)
        assert np.array_equal(conv, ov), (name, p)
        assert np.array_equal(corr, oc.astype(np.int64)), (name, p)


def test_hbm_adaptive_alpha_and_nonuniform_priors(gpu, oracle):
    from qldpc_fault_tolerance_amd.engine import DeviceBP

    code = codes.get_code("hgp_34_n225")
    synd = _synd(code.hx, 0.05, 200, seed=3)
    probs = np.linspace(0.01, 0.09, code.N)
    dec = DeviceBP(code.hx, probs, max_iter=30, ms_scaling_factor=0.0, precision=64, hbm=True)
    corr, iters, conv = dec.decode_batch(synd)
    oc, oi, ov = oracle.bp_decode_batch(code.hx, probs, 30, "minimum_sum", 0.0, synd, 64)
    assert np.array_equal(corr, oc) and np.array_equal(iters, oi) and np.array_equal(conv, ov)


@pytest.mark.parametrize("precision", [64, 32])
def test_hbm_config4_mc_matches_oracle(gpu, oracle, precision):
    """Config 4 forced onto the HBM engine: the data-error shot loop (staged pipeline around the
    engine-6 decoders) against the oracle's shot loop, shot for shot."""
    from qldpc_fault_tolerance_amd.engine import DeviceBP, DeviceMC

    code = codes.get_code("LP_Matg8_L30_Dmin20")
    n, p = code.N, 0.05
    mi = int(n / 10)
    dx = DeviceBP(code.hz, p, max_iter=mi, precision=precision, hbm=True)
    dz = DeviceBP(code.hx, p, max_iter=mi, precision=precision, hbm=True)
    S = 700
    res = DeviceMC(code, dx, dz).run(p / 2, p / 2, p / 2, seed=4242, shot_begin=77, shot_count=S,
                                     logical_mode="Total", per_shot=True)
    ref = oracle.mc_run(code, p / 2, p / 2, p / 2, seed=4242, shot_begin=77, shot_count=S, logical_mode="Total",
                        probs_x=p, probs_z=p, max_iter=mi, precision=precision, per_shot=True)
    assert np.array_equal(res.fail, ref["fail"])
    assert res.failures == ref["failures"]
    assert res.sector_iters == ref["sector_iters"] and res.sector_nonconv == ref["sector_nonconv"]


def test_st_decoder_class_default_precision_n1225(gpu, oracle):
    """ST_BP_Decoder_Class().GetDecoder on hgp_34_n1225_q3 with num_rep = 3 at its default (fp64)
    precision: the 1764 x 5439 space-time decoder runs in LDS on engine 3's tail layout (rows of
    4 chunks + one tail slot: 162 KB instead of 176 KB) and matches the oracle bit for bit,
    converged (p = 0.01) and at max_iter (p = 0.04)."""
    code = codes.get_code("hgp_34_n1225_q3")
    st = decoders.ST_BP_Decoder_Class(max_iter_ratio=10, bp_method="minimum_sum", ms_scaling_factor=0.625)
    dec = st.GetDecoder({"h": code.hx, "p_data": 0.01, "p_syndrome": 0.01, "num_rep": 3})
    g = dec.space_decoder.geometry()
    assert g["engine"] == 3 and g["lds_bytes"] <= 160 * 1024, g
    mi = int(code.N / 10)
    for p, B in ((0.01, 150), (0.04, 130), (0.025, 600)):
        rng = np.random.default_rng(17 + B)
        e = (rng.random((B, dec.ST_csr.n)) < p).astype(np.uint8)
        synd = dec.ST_csr.matvec(e).astype(np.uint8)
        corr, iters, conv = dec.space_decoder.decode_batch(synd)
        oc, oi, ov = oracle.bp_decode_batch(dec.ST_csr, dec.channel_probs, mi, "minimum_sum", 0.625, synd, 64)
        assert np.array_equal(iters, oi) and np.array_equal(conv, ov), p
        assert np.array_equal(corr, oc.astype(corr.dtype)), p
        if p == 0.01:
            out = dec.decode_batch(synd.reshape(B, 3, -1))
            assert np.array_equal(out, decoders.fold_space_time_correction(oc, code.N, code.hx.shape[0], 3))
        else:
            assert (~ov.astype(bool)).sum() > 0  # decodes that run to max_iter are covered


def test_st_tail_layout_adaptive_alpha_zero_prior(gpu, oracle):
    """Tail layout with ldpc's adaptive alpha (ms_scaling_factor = 0) and a zero prior (p = 0.5 on
    the syndrome-error columns): bit-exact incl. the signed zeros of the w domain."""
    from qldpc_fault_tolerance_amd.engine import DeviceBP

    code = codes.get_code("hgp_34_n1225_q3")
    csr = codes.space_time_csr(np.asarray(code.hx), 3)
    n = csr.n
    probs = np.full(n, 0.02)
    probs[-code.hx.shape[0]:] = 0.5
    dec = DeviceBP(csr, probs, max_iter=40, ms_scaling_factor=0.0, precision=64)
    assert dec.geometry()["engine"] == 3
    rng = np.random.default_rng(5)
    e = (rng.random((96, n)) < 0.02).astype(np.uint8)
    synd = csr.matvec(e).astype(np.uint8)
    corr, iters, conv = dec.decode_batch(synd)
    oc, oi, ov = oracle.bp_decode_batch(csr, probs, 40, "minimum_sum", 0.0, synd, 64)
    assert np.array_equal(iters, oi) and np.array_equal(conv, ov) and np.array_equal(corr, oc.astype(corr.dtype))


def test_st_decoder_hbm_forced_n1225(gpu, oracle):
    """The same space-time graph forced onto the HBM engine (engine 6) stays bit-exact."""
    from qldpc_fault_tolerance_amd.engine import DeviceBP

    code = codes.get_code("hgp_34_n1225_q3")
    st = decoders.ST_BP_Decoder_Class(max_iter_ratio=10, bp_method="minimum_sum", ms_scaling_factor=0.625)
    dec = st.GetDecoder({"h": code.hx, "p_data": 0.01, "p_syndrome": 0.01, "num_rep": 3})
    mi = int(code.N / 10)
    hb = DeviceBP(dec.ST_csr, dec.channel_probs, max_iter=mi, precision=64, hbm=True)
    assert hb.geometry()["engine"] == 6
    rng = np.random.default_rng(23)
    e = (rng.random((150, dec.ST_csr.n)) < 0.01).astype(np.uint8)
    synd = dec.ST_csr.matvec(e).astype(np.uint8)
    corr, iters, conv = hb.decode_batch(synd)
    oc, oi, ov = oracle.bp_decode_batch(dec.ST_csr, dec.channel_probs, mi, "minimum_sum", 0.625, synd, 64)
    assert np.array_equal(iters, oi) and np.array_equal(conv, ov) and np.array_equal(corr, oc.astype(corr.dtype))
