"""GPU parity: the HIP kernels (through the C ABI) against the CPU oracle.

Bit-exact bar (integer/byte outputs): corrections, iteration counts,
convergence flags, sampled errors and failure flags must be identical to the
oracle on the same inputs, in float64 (the reference arithmetic) and in float32
(the oracle's float32 restatement in the same operation order).
"""
import numpy as np
import pytest

from qldpc_fault_tolerance_amd import codes

pytestmark = pytest.mark.gpu


def _sample_synd(H, p, B, seed):
    rng = np.random.default_rng(seed)
    e = (rng.random((B, H.shape[1])) < p).astype(np.uint8)
    return (e.astype(np.int64) @ H.T.astype(np.int64) % 2).astype(np.uint8)


@pytest.mark.parametrize("precision", [64, 32])
@pytest.mark.parametrize("name", ["hgp_34_n225", "hgp_34_n1600", "LP_Matg8_L30_Dmin20", "rand40x120"])
def test_one_iteration_decode_matches_oracle(gpu, oracle, monkeypatch, precision, name):
    """max_iter = 1 min-sum decodes (the circuit loop's h1 rounds) run the first-min step kernel
    (qldpc_bp_decode_batch's one-iteration path): corrections, iterations and convergence equal the
    oracle and the engine's own kernels (QLDPC_BP1=0), with non-uniform and tied priors, alpha 0.625
    and ldpc's alpha = 0 schedule."""
    from qldpc_fault_tolerance_amd.engine import DeviceBP

    if name == "rand40x120":  # <= 64 checks: the thread-per-syndrome kernel
        g = np.random.default_rng(3)
        H = np.zeros((40, 120), np.uint8)
        for j in range(120):
            H[g.choice(40, 3, replace=False), j] = 1
        n = 120
    else:
        H = codes.get_code(name).hz
        n = H.shape[1]
    rng = np.random.default_rng(n + precision)
    pr = rng.uniform(0.01, 0.1, n)
    pr[::4] = pr[1]
    synd = _sample_synd(H, 0.05, 300, seed=precision)
    for alpha in (0.625, 0.0):
        c, i, v = DeviceBP(H, pr, max_iter=1, ms_scaling_factor=alpha, precision=precision).decode_batch(synd)
        oc, oi, ov = oracle.bp_decode_batch(H, pr, 1, "minimum_sum", alpha, synd, precision)
        assert np.array_equal(i, oi) and np.array_equal(v, ov) and np.array_equal(c, oc.astype(np.int64)), alpha
        monkeypatch.setenv("QLDPC_BP1", "0")
        c2, i2, v2 = DeviceBP(H, pr, max_iter=1, ms_scaling_factor=alpha, precision=precision).decode_batch(synd)
        monkeypatch.delenv("QLDPC_BP1")
        assert np.array_equal(c2, c) and np.array_equal(i2, i) and np.array_equal(v2, v), alpha


@pytest.mark.parametrize("precision", [64, 32])
@pytest.mark.parametrize("name,ratio", [("hgp_34_n225", 10), ("GenBicycleA2", 10), ("LP_Matg8_L16_Dmin12", 10)])
def test_decode_batch_matches_oracle(gpu, oracle, precision, name, ratio):
    from qldpc_fault_tolerance_amd.engine import DeviceBP

    code = codes.get_code(name)
    H = code.hz
    n = code.N
    max_iter = int(n / ratio)
    for p in (0.02, 0.06, 0.12):
        synd = _sample_synd(H, p, 400, seed=int(p * 1000) + precision)
        dec = DeviceBP(H, p * np.ones(n), max_iter=max_iter, bp_method="minimum_sum", ms_scaling_factor=0.625,
                       precision=precision)
        corr, iters, conv = dec.decode_batch(synd)
        ocorr, oiters, oconv = oracle.bp_decode_batch(H, p, max_iter, "minimum_sum", 0.625, synd, precision)
        assert np.array_equal(iters, oiters), (name, p)
        assert np.array_equal(conv, oconv), (name, p)
        assert np.array_equal(corr, ocorr.astype(np.int64)), (name, p)


@pytest.mark.parametrize("precision", [64, 32])
def test_decode_zero_priors_matches_oracle(gpu, oracle, precision):
    """Channel probabilities of exactly 0.5 (zero prior LLRs, zero messages): the engine-3
    negated message domain maps them to +0 (bp_reg.h w_prior); decisions must still match."""
    from qldpc_fault_tolerance_amd.engine import DeviceBP

    code = codes.get_code("hgp_34_n225")
    H = code.hz
    n = code.N
    rng = np.random.default_rng(11)
    for frac in (0.1, 1.0):
        probs = np.full(n, 0.05)
        probs[rng.random(n) < frac] = 0.5
        synd = _sample_synd(H, 0.05, 200, seed=int(frac * 10) + precision)
        synd[:5] = 0  # all-zero syndromes: messages that stay exactly zero
        dec = DeviceBP(H, probs, max_iter=25, ms_scaling_factor=0.625, precision=precision)
        corr, iters, conv = dec.decode_batch(synd)
        ocorr, oiters, oconv = oracle.bp_decode_batch(H, probs, 25, "minimum_sum", 0.625, synd, precision)
        assert np.array_equal(iters, oiters), frac
        assert np.array_equal(conv, oconv), frac
        assert np.array_equal(corr, ocorr.astype(np.int64)), frac


def test_decode_adaptive_alpha_matches_oracle(gpu, oracle):
    from qldpc_fault_tolerance_amd.engine import DeviceBP

    code = codes.get_code("hgp_34_n225")
    synd = _sample_synd(code.hx, 0.05, 300, seed=7)
    dec = DeviceBP(code.hx, 0.05, max_iter=30, ms_scaling_factor=0.0, precision=64)
    corr, iters, conv = dec.decode_batch(synd)
    ocorr, oiters, oconv = oracle.bp_decode_batch(code.hx, 0.05, 30, "minimum_sum", 0.0, synd, 64)
    assert np.array_equal(corr, ocorr) and np.array_equal(iters, oiters) and np.array_equal(conv, oconv)


@pytest.mark.parametrize("precision", [64, 32])
@pytest.mark.parametrize("name", ["hgp_34_n225", "hgp_34_n1600", "LP_Matg8_L30_Dmin20", "GenBicycleA1", "GenBicycleA3",
                                  "GenBicycleA4"])
def test_mc_per_shot_matches_oracle(gpu, oracle, precision, name):
    from qldpc_fault_tolerance_amd.engine import DeviceBP, DeviceMC

    code = codes.get_code(name)
    n = code.N
    mi = int(n / 10)
    p = 0.04
    px = py = pz = p / 2
    dx = DeviceBP(code.hz, (px + py) * np.ones(n), max_iter=mi, precision=precision)
    dz = DeviceBP(code.hx, (pz + py) * np.ones(n), max_iter=mi, precision=precision)
    if precision == 32:  # the register engine serves every config graph in fp32 (column degree <= 6)
        assert dx.geometry()["engine"] == 3
    mc = DeviceMC(code, dx, dz)
    S = 300 if n > 1000 else 1500
    res = mc.run(px, py, pz, seed=0x51D5EED0, shot_begin=12345, shot_count=S, logical_mode="Total", per_shot=True)
    ref = oracle.mc_run(code, px, py, pz, seed=0x51D5EED0, shot_begin=12345, shot_count=S, logical_mode="Total",
                        max_iter=mi, precision=precision, per_shot=True)
    assert np.array_equal(res.err, ref["err"])
    assert np.array_equal(res.iters, ref["iters"])
    assert np.array_equal(res.corr, ref["corr"])
    assert np.array_equal(res.fail, ref["fail"])
    assert res.shots == ref["shots"] == S
    assert res.failures == ref["failures"]
    assert res.sector_iters == ref["sector_iters"]
    assert res.sector_nonconv == ref["sector_nonconv"]


def test_mc_external_uniforms_matches_oracle(gpu, oracle):
    """External u stream (e.g. CPython random()) reproduces the reference split exactly."""
    from qldpc_fault_tolerance_amd.engine import DeviceBP, DeviceMC
    import random

    code = codes.get_code("hgp_34_n225")
    n = code.N
    p = 0.05
    random.seed(2024)
    S = 200
    u = np.array([[random.random() for _ in range(n)] for _ in range(S)])
    dx = DeviceBP(code.hz, p * np.ones(n), max_iter=22, precision=64)
    dz = DeviceBP(code.hx, p * np.ones(n), max_iter=22, precision=64)
    mc = DeviceMC(code, dx, dz)
    res = mc.run(p / 2, p / 2, p / 2, seed=0, shot_begin=0, shot_count=S, logical_mode="Total", uniforms=u,
                 per_shot=True)
    ref = oracle.mc_run(code, p / 2, p / 2, p / 2, seed=0, shot_begin=0, shot_count=S, logical_mode="Total",
                        max_iter=22, uniforms=u, per_shot=True)
    assert np.array_equal(res.err, ref["err"])
    assert np.array_equal(res.corr, ref["corr"])
    assert np.array_equal(res.fail, ref["fail"])


def test_mc_shard_invariance(gpu):
    """Counters over a shot range are identical however the range is split (multi-GPU invariant)."""
    from qldpc_fault_tolerance_amd.engine import DeviceBP, DeviceMC

    code = codes.get_code("hgp_34_n225")
    n = code.N
    p = 0.05
    dx = DeviceBP(code.hz, p * np.ones(n), max_iter=22, precision=32)
    mc = DeviceMC(code, dx, None)
    whole = mc.run(p / 2, p / 2, p / 2, seed=99, shot_begin=1000, shot_count=6000, logical_mode="X")
    parts = None
    for b, c in [(1000, 1500), (2500, 2500), (5000, 2000)]:
        r = mc.run(p / 2, p / 2, p / 2, seed=99, shot_begin=b, shot_count=c, logical_mode="X")
        parts = r if parts is None else parts.merge(r)
    assert whole.failures == parts.failures
    assert whole.sector_iters == parts.sector_iters
    assert np.array_equal(whole.iter_hist, parts.iter_hist)
