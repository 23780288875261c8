"""GPU parity of the fp64 space-time "m2 in slot" family (engine id 111313, round 6) beyond config 5.

The family decodes the stacked space-time graphs of ``GetSpaceTimeCheckMat`` (``src/Decoders_SpaceTime.py:
179-194``) with 1024-thread workgroups; its host plan (``qldpc_hip.hip`` ``st_plan``) sorts the columns by
degree, runs the leading waves of the first two variable slots one edge slot narrower (narrow waves) and
places the logical waves on the SIMDs.  Config 5 (hgp_34_n1225_q3, three rounds: 6 variable slots) is
replayed against the reference's histories in ``test_gpu_golden.py``; here a second graph with another
slot structure (hgp_34_n1600 over two rounds: 1536 x 4736, 5 variable slots, 768 degree-1 and 768
degree-2 measurement columns; an fp64 image of 117 KB that ran on engine 2 before round 6) and config
5's graph decode i.i.d. syndromes bit-exactly against the oracle, and every plan switch (narrow waves,
SIMD placement) leaves the outputs unchanged.  hgp_34_n1225_q3 over two rounds (4 variable slots) takes
the two-word tail family (engine id 1013; the one-word family is built for 5 and 6 slots); hgp_34_n625
over three rounds and GenBicycleA4 over two (rows of 8: an empty tail slot) run 512-thread workgroups,
two decodes per CU; GenBicycleA3 over five rounds (rows of 8) the two-word tail family.
"""
import numpy as np
import pytest

from qldpc_fault_tolerance_amd import codes

pytestmark = pytest.mark.gpu


def _synd(H, p, B, seed):
    rng = np.random.default_rng(seed)
    e = (rng.random((B, H.n)) < p).astype(np.int64)
    Hd = np.zeros((H.m, H.n), np.int64)
    Hd[np.repeat(np.arange(H.m), np.diff(H.row_ptr)), H.col_idx] = 1
    return (e @ Hd.T % 2).astype(np.uint8), Hd.astype(np.uint8)


@pytest.mark.parametrize("name,t0,kid,tb,vpl", [
    ("hgp_34_n1600", 2, 111313, 1024, 5), ("hgp_34_n1225_q3", 3, 111313, 1024, 6), ("hgp_34_n1225_q3", 2, 1013, 1024, 4),
    # 512-thread geometries (two decodes per CU) and rows of 8 (an empty tail slot per row)
    ("hgp_34_n625", 3, 111313, 512, 6), ("GenBicycleA4", 2, 111313, 512, 6), ("GenBicycleA3", 5, 1013, 1024, 4)])
def test_space_time_one_word_family_matches_oracle(gpu, oracle, monkeypatch, name, t0, kid, tb, vpl):
    from qldpc_fault_tolerance_amd.engine import DeviceBP

    code = codes.get_code(name)
    Hst = codes.space_time_csr(code.hz, t0)
    n = code.N
    mi = int(n / 10)
    for p, B in ((0.01, 192), (0.05, 96)):
        synd, Hd = _synd(Hst, p, B, seed=int(p * 1000) + t0)
        probs = np.hstack([p * np.ones(n), p * np.ones(code.hz.shape[0])] * t0)
        dec = DeviceBP(Hst, probs, max_iter=mi, precision=64)
        g = dec.geometry()
        assert (g["engine"], g["kernel_id"], g["threads"], g["vars_per_thread"]) == (3, kid, tb, vpl), g
        c, i, v = dec.decode_batch(synd)
        oc, oi, ov = oracle.bp_decode_batch(Hd, probs, mi, "minimum_sum", 0.625, synd, 64)
        assert np.array_equal(i, oi) and np.array_equal(v, ov), (name, p)
        assert np.array_equal(c, oc.astype(np.int64)), (name, p)
        # the plan switches: no narrow waves (the pre-round-6 slot order), waves in order
        for env in ({"QLDPC_NW": "0"}, {"QLDPC_NW_BAL": "0"}):
            for k, val in env.items():
                monkeypatch.setenv(k, val)
            d2 = DeviceBP(Hst, probs, max_iter=mi, precision=64)
            assert d2.geometry()["kernel_id"] == kid
            c2, i2, v2 = d2.decode_batch(synd)
            for k in env:
                monkeypatch.delenv(k)
            assert np.array_equal(c2, c) and np.array_equal(i2, i) and np.array_equal(v2, v), (name, p, env)


def test_graph_without_a_compiled_engine3_variant_falls_back_to_hbm(gpu, oracle):
    """GenBicycleA4 over five rounds in fp32 (2555 x 7665, rows of 8): engine 3's dword-scaled fp32
    family is compiled for 3-7 variables per thread and this geometry needs 8 (round 6: creation failed
    with "no kernel variant"); the decoder now falls back to the HBM-resident engine, bit-exact against
    the oracle's fp32 restatement."""
    from qldpc_fault_tolerance_amd.engine import DeviceBP

    code = codes.get_code("GenBicycleA4")
    Hst = codes.space_time_csr(code.hz, 5)
    n, p = code.N, 0.01
    probs = np.hstack([p * np.ones(n), p * np.ones(code.hz.shape[0])] * 5)
    dec = DeviceBP(Hst, probs, max_iter=int(n / 10), precision=32)
    assert dec.geometry()["engine"] == 6, dec.geometry()
    synd, Hd = _synd(Hst, p, 64, seed=9)
    c, i, v = dec.decode_batch(synd)
    oc, oi, ov = oracle.bp_decode_batch(Hd, probs, int(n / 10), "minimum_sum", 0.625, synd, 32)
    assert np.array_equal(i, oi) and np.array_equal(v, ov) and np.array_equal(c, oc.astype(np.int64))
