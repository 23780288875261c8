"""The fp64 one-slot families against the oracle: "m2 in slot" (engine id 11103, bp_reg.h eng_m2s,
the default for the headline graphs), "c2v in slot" (31103, eng_c2s, QLDPC_C2S=1) and m2s with
variable-major V slots (40103, eng_m2v, QLDPC_M2V=1).

The headline graphs (hgp_34_n1600 hz / hx: rows of exactly 7, column degrees 3 / 4 with the
degree-3 variables filling 4 whole slots of 256 lanes) run in float64 with rows of 3 chunks + a
tail slot and 3 workgroups per CU.  c2s: the check phase writes every edge's c2v into the row's
slots (46.2 KB image, no check-state array); m2s: one-word check state {m1 | parity} and m2 |
parity in the argmin edge's V slot (52.3 KB).  Bit-exact bar as every other engine: corrections,
iteration counts and convergence flags identical to the oracle's float64 restatement of ldpc; the
three families (c2s, m2s, two-word QLDPC_M2S=0) identical on the same inputs.
"""
import os

import numpy as np
import pytest

from qldpc_fault_tolerance_amd import codes

pytestmark = pytest.mark.gpu


def _synd(H, p, B, seed):
    rng = np.random.default_rng(seed)
    e = (rng.random((B, H.shape[1])) < p).astype(np.uint8)
    return (e.astype(np.int64) @ H.T.astype(np.int64) % 2).astype(np.uint8)


def _experimental():
    from qldpc_fault_tolerance_amd import _native

    return _native.experimental_families()


def _need(fam):
    """c2s / m2v are measured-and-not-kept families, compiled only into experimental builds."""
    if fam in ("c2s", "m2v") and not _experimental():
        pytest.skip(f"{fam} family not in this build (QLDPC_EXPERIMENTAL=0)")


def _dec(H, probs, mi, alpha=0.625, m2s=True, vpl=0, c2s=False, m2v=False):
    from qldpc_fault_tolerance_amd.engine import DeviceBP

    env = {"QLDPC_M2S": "1" if m2s else "0", "QLDPC_C2S": "1" if c2s else "0", "QLDPC_M2V": "1" if m2v else "0"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return DeviceBP(H, probs, max_iter=mi, ms_scaling_factor=alpha, precision=64, vars_per_thread=vpl)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def test_headline_graphs_select_m2s_family(gpu):
    code = codes.get_code("hgp_34_n1600")
    exp = _experimental()
    for H in (code.hz, code.hx):
        g1 = _dec(H, 0.06, 160).geometry()
        assert (g1["engine"], g1["kernel_id"], g1["row_chunks"], g1["threads"], g1["vars_per_thread"]) == \
            (3, 11103, 3, 256, 7), g1
        assert g1["degree3_slots"] == 4 and g1["lds_bytes"] * 3 <= 160 * 1024 and g1["blocks_per_cu"] == 3, g1
        g0 = _dec(H, 0.06, 160, m2s=False).geometry()
        assert g0["kernel_id"] == 103 and g0["blocks_per_cu"] == 2, g0
        g = _dec(H, 0.06, 160, c2s=True).geometry()  # opt-in honoured only where the family is built
        assert g["kernel_id"] == (31103 if exp else 11103), g
        if exp:
            assert g["blocks_per_cu"] == 3 and g1["lds_bytes"] > g["lds_bytes"], (g1, g)
        g2 = _dec(H, 0.06, 160, m2v=True).geometry()  # variable-major V slots
        assert g2["kernel_id"] == (40103 if exp else 11103) and g2["blocks_per_cu"] == 3, g2
    # outside the envelope (mixed-degree slots: n225's 144 degree-3 variables over 64 lanes) -> two-word family
    assert _dec(codes.get_code("hgp_34_n225").hz, 0.05, 22).geometry()["kernel_id"] not in (11103, 31103)


@pytest.mark.parametrize("sector", ["hz", "hx"])
@pytest.mark.parametrize("p", [0.02, 0.06, 0.12])
def test_m2s_decode_matches_oracle(gpu, oracle, sector, p):
    code = codes.get_code("hgp_34_n1600")
    H = getattr(code, sector)
    B = 512
    synd = _synd(H, p, B, seed=int(p * 1e4) + (sector == "hx"))
    synd[:3] = 0
    c, i, v = _dec(H, p, 160).decode_batch(synd)
    oc, oi, ov = oracle.bp_decode_batch(H, p, 160, "minimum_sum", 0.625, synd, 64)
    assert np.array_equal(i, oi) and np.array_equal(v, ov) and np.array_equal(c, oc.astype(np.int64))
    for kw in ({"m2s": False}, {"c2s": True}, {"m2v": True}):
        c0, i0, v0 = _dec(H, p, 160, **kw).decode_batch(synd)
        assert np.array_equal(c, c0) and np.array_equal(i, i0) and np.array_equal(v, v0), kw


@pytest.mark.parametrize("fam", ["c2s", "m2s", "m2v"])
def test_m2s_adaptive_alpha_and_zero_priors_match_oracle(gpu, oracle, fam):
    """Adaptive alpha and all-zero priors on the c2s / m2s families; non-uniform priors take the
    two-word family (all keep one prior in SGPRs: QLDPC_M2S_UNIL)."""
    _need(fam)
    c2s, m2v = fam == "c2s", fam == "m2v"
    code = codes.get_code("hgp_34_n1600")
    H = code.hz
    synd = _synd(H, 0.05, 256, seed=5)
    c, i, v = _dec(H, 0.05, 60, alpha=0.0, c2s=c2s, m2v=m2v).decode_batch(synd)
    oc, oi, ov = oracle.bp_decode_batch(H, 0.05, 60, "minimum_sum", 0.0, synd, 64)
    assert np.array_equal(c, oc.astype(np.int64)) and np.array_equal(i, oi) and np.array_equal(v, ov)
    # every prior zero (p = 0.5): messages that are exactly +-0 on the one-prior kernels
    dec = _dec(H, 0.5, 12, c2s=c2s, m2v=m2v)
    assert dec.geometry()["kernel_id"] == {"c2s": 31103, "m2s": 11103, "m2v": 40103}[fam]
    c, i, v = dec.decode_batch(synd)
    oc, oi, ov = oracle.bp_decode_batch(H, 0.5, 12, "minimum_sum", 0.625, synd, 64)
    assert np.array_equal(c, oc.astype(np.int64)) and np.array_equal(i, oi) and np.array_equal(v, ov)
    # non-uniform priors (some zero): the m2s kernels hold one prior, so the two-word family serves
    rng = np.random.default_rng(3)
    probs = np.full(code.N, 0.04)
    probs[rng.random(code.N) < 0.3] = 0.5
    dec = _dec(H, probs, 40, c2s=c2s, m2v=m2v)
    assert dec.geometry()["kernel_id"] == 103
    c, i, v = dec.decode_batch(synd)
    oc, oi, ov = oracle.bp_decode_batch(H, probs, 40, "minimum_sum", 0.625, synd, 64)
    assert np.array_equal(c, oc.astype(np.int64)) and np.array_equal(i, oi) and np.array_equal(v, ov)


@pytest.mark.parametrize("fam", ["c2s", "m2s", "m2v"])
def test_m2s_fused_mc_matches_oracle_per_shot(gpu, oracle, fam):
    from qldpc_fault_tolerance_amd.engine import DeviceMC

    _need(fam)
    code = codes.get_code("hgp_34_n1600")
    n, p, S = code.N, 0.07, 400
    c2s, m2v = fam == "c2s", fam == "m2v"
    dx, dz = _dec(code.hz, p, 160, c2s=c2s, m2v=m2v), _dec(code.hx, p, 160, vpl=7, c2s=c2s, m2v=m2v)
    assert dx.geometry()["kernel_id"] == dz.geometry()["kernel_id"] == {"c2s": 31103, "m2s": 11103, "m2v": 40103}[fam]
    res = DeviceMC(code, dx, dz).run(p / 2, p / 2, p / 2, 0x51D5EED2, 777, S, "Total", per_shot=True)
    ref = oracle.mc_run(code, p / 2, p / 2, p / 2, seed=0x51D5EED2, shot_begin=777, shot_count=S, logical_mode="Total",
                        max_iter=160, precision=64, per_shot=True)
    for k in ("err", "iters", "corr", "fail"):
        assert np.array_equal(getattr(res, k), ref[k]), k
    assert res.failures == ref["failures"] and res.sector_iters == ref["sector_iters"]


def _biregular(m, n, dc, dv, seed):
    """A random (dv, dc)-regular m x n parity-check matrix (configuration model, no double edges)."""
    rng = np.random.default_rng(seed)
    while True:
        stubs = np.repeat(np.arange(n), dv)
        rng.shuffle(stubs)
        H = np.zeros((m, n), np.uint8)
        ok = True
        for i in range(m):
            for j in stubs[i * dc:(i + 1) * dc]:
                ok = ok and not H[i, j]
                H[i, j] = 1
        if ok:
            return H


def asymmetric_hgp():
    """HGP of a (3,4)-regular 6x8 h1 and a rank-deficient (3,3)-regular 8x8 h2: hx is all
    degree 3 (rows of 7), hz has 64 degree-3 and 48 degree-4 columns (rows of 6).  With 4 variables per
    thread (64 lanes) both sectors qualify for the one-word fp64 families, with different degree-3
    slot counts (hx 4, hz 1)."""
    from qldpc_fault_tolerance_amd import gf2

    h2 = next(h for h in (_biregular(8, 8, 3, 3, 100 + s) for s in range(64)) if gf2.rank(h) < 8)
    return codes.hgp(_biregular(6, 8, 4, 3, 7), h2, name="hgp_asym_112")


@pytest.mark.parametrize("fam", ["m2s", "c2s"])
def test_m2s_fused_mc_asymmetric_sectors_matches_oracle(gpu, oracle, fam):
    """Sectors whose degree-3 slot counts differ cannot share one compile-time D3K kernel (a
    degree-3 variable would run the 4-edge path and read the shared dummy V slot): the MC must
    route them to the staged pipeline and stay bit-exact."""
    from qldpc_fault_tolerance_amd.engine import DeviceMC

    _need(fam)
    code = asymmetric_hgp()
    assert code.N == 112 and code.K > 0
    p, S, mi = 0.06, 600, 20
    dx, dz = _dec(code.hz, p, mi, vpl=4, c2s=fam == "c2s"), _dec(code.hx, p, mi, vpl=4, c2s=fam == "c2s")
    gx, gz = dx.geometry(), dz.geometry()
    assert gx["kernel_id"] == gz["kernel_id"] == 11103 or fam == "c2s", (gx, gz)
    assert (gx["degree3_slots"], gz["degree3_slots"]) == (1, 4), (gx, gz)
    res = DeviceMC(code, dx, dz).run(p / 2, p / 2, p / 2, 0x51D5EED3, 11, S, "Total", per_shot=True)
    ref = oracle.mc_run(code, p / 2, p / 2, p / 2, seed=0x51D5EED3, shot_begin=11, shot_count=S, logical_mode="Total",
                        max_iter=mi, precision=64, per_shot=True)
    for k in ("err", "iters", "corr", "fail"):
        assert np.array_equal(getattr(res, k), ref[k]), k
    assert res.failures == ref["failures"] and res.sector_iters == ref["sector_iters"]
