"""The fp64 "m2 in slot" family for rows of 8 and column degree 5 (engine id 10103,
kern_r_f64_m2s8.hip): config 4's LP_Matg8_L30_Dmin20 (450 x 1020, rows of 8,
750 degree-3 and 270 degree-5 columns) in float64 with the one-word check state: 256 threads x 4
variable slots, 2 degree-3 slots, and the 238 degree-3 variables of the third slot (shared with the
degree-5 class) keep PRIVATE dummy V slots for their two missing edges (c2v = +-0 from the zero CS
entry; w-domain sums are never -0, so every message stays bit-exact).

Bit-exact bar as every other engine: corrections, iteration counts and convergence flags
identical to the oracle's float64 restatement of ldpc (``src/Decoders.py:80-84``) and to the
two-word family (``QLDPC_M2S8=0``) on the same inputs; the fused MC per shot identical to the
oracle's ``_single_run`` restatement.
"""
import os

import numpy as np
import pytest

from qldpc_fault_tolerance_amd import codes

pytestmark = pytest.mark.gpu

LP = "LP_Matg8_L30_Dmin20"


def _synd(H, p, B, seed):
    rng = np.random.default_rng(seed)
    e = (rng.random((B, H.shape[1])) < p).astype(np.uint8)
    return (e.astype(np.int64) @ H.T.astype(np.int64) % 2).astype(np.uint8)


def _dec(H, probs, mi, alpha=0.625, m2s8=True, pk=False):
    """pk: the packed-address variant (engine id 10203, QLDPC_M2S8_PK=1, 4 workgroups per CU)."""
    from qldpc_fault_tolerance_amd.engine import DeviceBP

    env = {"QLDPC_M2S8": "1" if m2s8 else "0", "QLDPC_M2S8_PK": "1" if pk else "0"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return DeviceBP(H, probs, max_iter=mi, ms_scaling_factor=alpha, precision=64)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


FAM = {False: 10103, True: 10203}


def ragged_35(seed=11):
    """600 degree-3 and 200 degree-5 columns over 400 rows of 5-8 edges: rows with padding slots, 88
    degree-3 variables with private dummy slots in the slot shared with the degree-5 class, a last
    slot of 32 degree-5 variables (waves 1-3 skip it)."""
    rng = np.random.default_rng(seed)
    n3, n5, m = 600, 200, 400
    while True:
        stubs = np.concatenate([np.repeat(np.arange(n3), 3), np.repeat(np.arange(n3, n3 + n5), 5)])
        rng.shuffle(stubs)
        H = np.zeros((m, n3 + n5), np.uint8)
        cap = np.zeros(m, int)
        ok = True
        for j in stubs:
            free = np.flatnonzero((cap < 8) & (H[:, j] == 0))
            if free.size == 0:
                ok = False
                break
            i = free[np.argmin(cap[free] + rng.random(free.size))]
            H[i, j] = 1
            cap[i] += 1
        if ok and cap.min() >= 5:
            return H


@pytest.mark.parametrize("pk", [False, True])
def test_lp30_selects_m2s8_family(gpu, pk):
    code = codes.get_code(LP)
    for H in (code.hz, code.hx):
        g = _dec(H, 0.06, 102, pk=pk).geometry()
        assert (g["engine"], g["kernel_id"], g["row_chunks"], g["threads"], g["vars_per_thread"]) == \
            (3, FAM[pk], 4, 256, 4), g
        assert g["degree3_slots"] == 2 and g["blocks_per_cu"] >= (4 if pk else 3), g
        g0 = _dec(H, 0.06, 102, m2s8=False).geometry()
        # (the one-word state saves 8 B per check; the private dummy slots cost 16 B per degree-3
        # variable of the shared slot: about the same image, but 168 instead of 256 VGPRs)
        assert g0["kernel_id"] == 103 and g["lds_bytes"] <= 40 * 1024, (g, g0)


@pytest.mark.parametrize("pk", [False, True])
@pytest.mark.parametrize("sector", ["hz", "hx"])
@pytest.mark.parametrize("p", [0.02, 0.06, 0.12])
def test_m2s8_decode_matches_oracle(gpu, oracle, sector, p, pk):
    H = getattr(codes.get_code(LP), sector)
    synd = _synd(H, p, 512, seed=int(p * 1e4) + (sector == "hx"))
    synd[:3] = 0
    dec = _dec(H, p, 102, pk=pk)
    assert dec.geometry()["kernel_id"] == FAM[pk]
    c, i, v = dec.decode_batch(synd)
    oc, oi, ov = oracle.bp_decode_batch(H, p, 102, "minimum_sum", 0.625, synd, 64)
    assert np.array_equal(i, oi) and np.array_equal(v, ov) and np.array_equal(c, oc.astype(np.int64))
    c0, i0, v0 = _dec(H, p, 102, m2s8=False).decode_batch(synd)
    assert np.array_equal(c, c0) and np.array_equal(i, i0) and np.array_equal(v, v0)


@pytest.mark.parametrize("pk", [False, True])
def test_m2s8_ragged_rows_match_oracle(gpu, oracle, pk):
    H = ragged_35()
    g = _dec(H, 0.05, 80, pk=pk).geometry()
    assert (g["kernel_id"], g["vars_per_thread"], g["degree3_slots"]) == (FAM[pk], 4, 2), g
    for p, seed in ((0.03, 1), (0.08, 2)):
        synd = _synd(H, p, 384, seed)
        c, i, v = _dec(H, p, 80, pk=pk).decode_batch(synd)
        oc, oi, ov = oracle.bp_decode_batch(H, p, 80, "minimum_sum", 0.625, synd, 64)
        assert np.array_equal(i, oi) and np.array_equal(v, ov) and np.array_equal(c, oc.astype(np.int64)), p


@pytest.mark.parametrize("pk", [False, True])
def test_m2s8_adaptive_alpha_and_zero_priors_match_oracle(gpu, oracle, pk):
    H = codes.get_code(LP).hz
    synd = _synd(H, 0.05, 256, seed=5)
    c, i, v = _dec(H, 0.05, 60, alpha=0.0, pk=pk).decode_batch(synd)
    oc, oi, ov = oracle.bp_decode_batch(H, 0.05, 60, "minimum_sum", 0.0, synd, 64)
    assert np.array_equal(c, oc.astype(np.int64)) and np.array_equal(i, oi) and np.array_equal(v, ov)
    dec = _dec(H, 0.5, 12, pk=pk)  # every prior zero: messages that are exactly +-0
    assert dec.geometry()["kernel_id"] == FAM[pk]
    c, i, v = dec.decode_batch(synd)
    oc, oi, ov = oracle.bp_decode_batch(H, 0.5, 12, "minimum_sum", 0.625, synd, 64)
    assert np.array_equal(c, oc.astype(np.int64)) and np.array_equal(i, oi) and np.array_equal(v, ov)
    probs = np.full(H.shape[1], 0.04)  # non-uniform priors: the two-word family serves
    probs[::7] = 0.5
    assert _dec(H, probs, 40).geometry()["kernel_id"] == 103


@pytest.mark.parametrize("pk", [False, True])
def test_m2s8_fused_mc_matches_oracle_per_shot(gpu, oracle, pk):
    from qldpc_fault_tolerance_amd.engine import DeviceMC

    code = codes.get_code(LP)
    p, S, mi = 0.06, 400, 102
    dx, dz = _dec(code.hz, p, mi, pk=pk), _dec(code.hx, p, mi, pk=pk)
    assert dx.geometry()["kernel_id"] == dz.geometry()["kernel_id"] == FAM[pk]
    res = DeviceMC(code, dx, dz).run(p / 2, p / 2, p / 2, 0x51D5EED4, 4321, S, "Total", per_shot=True)
    ref = oracle.mc_run(code, p / 2, p / 2, p / 2, seed=0x51D5EED4, shot_begin=4321, shot_count=S, logical_mode="Total",
                        max_iter=mi, precision=64, per_shot=True)
    for k in ("err", "iters", "corr", "fail"):
        assert np.array_equal(getattr(res, k), ref[k]), k
    assert res.failures == ref["failures"] and res.sector_iters == ref["sector_iters"]
    assert 0 < res.failures < S


@pytest.mark.parametrize("name,tb,vpl", [("LP_Matg8_L16_Dmin12", 128, 5), ("LP_Matg8_L21_Dmin16", 192, 5)])
def test_m2s8_small_lp_codes_at_fewer_threads_match_oracle(gpu, oracle, monkeypatch, name, tb, vpl):
    """The Threshold notebook's smaller lifted-product codes (544 / 714 columns; they came out at 256
    threads x 3 variables, below the family's 4-6, and ran on engine 2 before round 6) run the rows-of-8
    family with packed addresses at 128 / 192 threads x 5 variables: bit-exact against the oracle and
    against their old route (QLDPC_M2S8_SMALL=0)."""
    code = codes.get_code(name)
    for sector in ("hz", "hx"):
        H = getattr(code, sector)
        for p, seed in ((0.03, 1), (0.08, 2)):
            synd = _synd(H, p, 384, seed)
            dec = _dec(H, p, 54, pk=True)
            g = dec.geometry()
            assert (g["engine"], g["kernel_id"], g["threads"], g["vars_per_thread"]) == \
                (3, FAM[vpl <= 5], tb, vpl), g
            c, i, v = dec.decode_batch(synd)
            oc, oi, ov = oracle.bp_decode_batch(H, p, 54, "minimum_sum", 0.625, synd, 64)
            assert np.array_equal(i, oi) and np.array_equal(v, ov) and np.array_equal(c, oc.astype(np.int64)), p
            monkeypatch.setenv("QLDPC_M2S8_SMALL", "0")
            d0 = _dec(H, p, 54, pk=True)
            monkeypatch.delenv("QLDPC_M2S8_SMALL")
            assert d0.geometry()["engine"] == 2
            c0, i0, v0 = d0.decode_batch(synd)
            assert np.array_equal(c, c0) and np.array_equal(i, i0) and np.array_equal(v, v0), p


@pytest.mark.parametrize("name,vpl", [("LP_Matg8_L16_Dmin12", 4), ("LP_Matg8_L21_Dmin16", 5), ("LP_Matg8_L30_Dmin20", 6)])
def test_lp_h_identity_graphs_on_the_degree5_family_match_oracle(gpu, oracle, monkeypatch, name, vpl):
    """[h | I] of the Threshold notebook's lifted-product codes (CodeSimulator_Phenon's decoder1 graph,
    ``src/Simulators.py:189-250``: rows of 9, columns of degree 1 / 3 / 5) on the two-word degree-5
    family with 5-chunk rows at 256 threads (round 6; engine 2 before): bit-exact against the oracle and
    the old route (QLDPC_F64W=0)."""
    from qldpc_fault_tolerance_amd.engine import DeviceBP

    h = codes.get_code(name).hz
    H = np.hstack([h, np.eye(h.shape[0], dtype=np.uint8)])
    mi = int(h.shape[1] / 30)
    for p, seed in ((0.02, 3), (0.06, 4)):
        synd = _synd(H, p, 384, seed)
        dec = DeviceBP(H, p * np.ones(H.shape[1]), max_iter=mi, precision=64)
        g = dec.geometry()
        assert (g["engine"], g["kernel_id"], g["threads"], g["vars_per_thread"], g["row_chunks"]) == \
            (3, 103, 256, vpl, 5), g
        c, i, v = dec.decode_batch(synd)
        oc, oi, ov = oracle.bp_decode_batch(H, p, mi, "minimum_sum", 0.625, synd, 64)
        assert np.array_equal(i, oi) and np.array_equal(v, ov) and np.array_equal(c, oc.astype(np.int64)), p
        monkeypatch.setenv("QLDPC_F64W", "0")
        monkeypatch.setenv("QLDPC_D5_256", "0")
        d0 = DeviceBP(H, p * np.ones(H.shape[1]), max_iter=mi, precision=64)
        monkeypatch.delenv("QLDPC_F64W")
        monkeypatch.delenv("QLDPC_D5_256")
        assert d0.geometry()["engine"] == 2
        c0, i0, v0 = d0.decode_batch(synd)
        assert np.array_equal(c, c0) and np.array_equal(i, i0) and np.array_equal(v, v0), p
