"""CPU tests of the BP+OSD post-processing stage.

The native OSD (csrc/osd.hip: host code in libqldpc_hip.so, xor-basis
elimination + linear candidate updates) is compared bit-for-bit with the
oracle's literal restatement of ldpc 0.1's OSD (oracle/oracle.py osd_decode:
Neal LU with column swaps, one substitution per candidate) on posteriors from
the oracle's soft-output min-sum.  The reference's BPOSD_Decoder uses
osd_method="osd_e", osd_order=10 (SingleShotDecodingDemo / Threshold notebooks);
parity unpinned against ldpc/bposd themselves (absent), see DESIGN.md.
"""
import numpy as np
import pytest

from qldpc_fault_tolerance_amd import codes, gf2
from qldpc_fault_tolerance_amd.engine import HostOSD


def _syndromes(H, p, B, seed):
    rng = np.random.default_rng(seed)
    e = (rng.random((B, H.shape[1])) < p).astype(np.uint8)
    return (e.astype(np.int64) @ H.T.astype(np.int64) % 2).astype(np.uint8), e


@pytest.fixture(scope="module")
def n225():
    return codes.get_code("hgp_34_n225").hz.astype(np.uint8)


@pytest.mark.parametrize("method,order", [("osd_0", 0), ("osd_e", 0), ("osd_e", 3), ("osd_e", 6),
                                          ("osd_cs", 4), ("osd_cs", 7)])
def test_native_osd_matches_oracle_on_bp_posteriors(oracle, n225, method, order):
    H = n225
    p = 0.09
    synd, _ = _syndromes(H, p, 24, seed=11 + order)
    probs = np.full(H.shape[1], p)
    corr, _, conv, post = oracle.bp_decode_batch_soft(H, probs, 22, 0.625, synd)
    assert (~conv).sum() >= 4, "the case must exercise OSD"
    osd = HostOSD(H, probs, osd_method=method, osd_order=order)
    assert osd.rank == gf2.rank(H)
    o0, ow = osd.decode_batch(synd, post, conv, corr, threads=3)
    for b in range(synd.shape[0]):
        if conv[b]:
            assert np.array_equal(ow[b], corr[b]) and np.array_equal(o0[b], corr[b])
            continue
        r0, rw = oracle.osd_decode(H, probs, synd[b], post[b], method, order)
        assert np.array_equal(o0[b], r0), b
        assert np.array_equal(ow[b], rw), b
        # every OSD output satisfies the syndrome (H is consistent for sampled errors)
        assert np.array_equal(H.astype(np.int64) @ ow[b] % 2, synd[b])
        assert ow[b].sum() <= o0[b].sum()


def test_native_osd_ties_and_nonuniform_priors(oracle, n225):
    """Integer-valued posteriors (many ties: the stable sort decides) and
    non-uniform channel probabilities (soft weight summed in index order)."""
    H = n225
    rng = np.random.default_rng(5)
    synd, _ = _syndromes(H, 0.08, 12, seed=3)
    post = rng.integers(-2, 3, size=(12, H.shape[1])).astype(np.float64)
    probs = rng.uniform(0.01, 0.2, size=H.shape[1])
    for method, order in (("osd_e", 5), ("osd_cs", 5)):
        osd = HostOSD(H, probs, osd_method=method, osd_order=order)
        o0, ow = osd.decode_batch(synd, post)
        for b in range(12):
            r0, rw = oracle.osd_decode(H, probs, synd[b], post[b], method, order)
            assert np.array_equal(o0[b], r0) and np.array_equal(ow[b], rw), (method, b)


def test_native_osd_rank_deficient_space_time_graph(oracle):
    """The ST graph of a small code (rank-deficient stacked checks)."""
    h = codes.get_code("hgp_34_n225").hz.astype(np.uint8)[:36]
    H = codes.space_time_csr(h, 2).to_dense().astype(np.uint8)
    synd, _ = _syndromes(H, 0.05, 10, seed=9)
    rng = np.random.default_rng(1)
    post = rng.normal(size=(10, H.shape[1]))
    probs = np.full(H.shape[1], 0.05)
    osd = HostOSD(H, probs, osd_method="osd_e", osd_order=4)
    assert osd.rank == gf2.rank(H)
    o0, ow = osd.decode_batch(synd, post)
    for b in range(10):
        r0, rw = oracle.osd_decode(H, probs, synd[b], post[b], "osd_e", 4)
        assert np.array_equal(o0[b], r0) and np.array_equal(ow[b], rw), b


def test_osd_order_clipped_and_errors(n225):
    H = n225
    k = H.shape[1] - gf2.rank(H)
    osd = HostOSD(H, 0.05, osd_method="osd_e", osd_order=3)
    assert osd.rank + k == H.shape[1]
    with pytest.raises(ValueError):
        HostOSD(H, 0.05, osd_method="nope")
    from qldpc_fault_tolerance_amd._native import QldpcError

    with pytest.raises(QldpcError):
        HostOSD(H, 0.05, osd_method="osd_e", osd_order=40)
    with pytest.raises(QldpcError):
        HostOSD(H, 1.5)
    # empty batch
    o0, ow = osd.decode_batch(np.zeros((0, H.shape[0]), np.uint8), np.zeros((0, H.shape[1])))
    assert o0.shape == (0, H.shape[1])


@pytest.mark.parametrize("method,order", [("osd_e", 7), ("osd_cs", 8), ("osd_0", 0), ("osd_e", 4)])
def test_c_osd_restatement_matches_python_restatement(oracle, n225, method, order):
    """oracle_osd_decode_batch (C, bit-vector rows) == osd_decode (literal Python) on n225
    BP posteriors, tied integer posteriors and non-uniform priors: the C restatement is then
    trusted as the checker at n1600 OSD-E(10), where the Python loops are too slow."""
    H = n225
    p = 0.09
    synd, _ = _syndromes(H, p, 6, seed=23 + order)
    probs = np.full(H.shape[1], p)
    _, _, conv, post = oracle.bp_decode_batch_soft(H, probs, 22, 0.625, synd)
    rng = np.random.default_rng(order)
    cases = [(synd, post, probs),
             (synd[:4], rng.integers(-2, 3, size=(4, H.shape[1])).astype(np.float64), probs),
             (synd[:4], post[:4], rng.uniform(0.01, 0.2, size=H.shape[1]))]
    for s, ps, pr in cases:
        c0, cw = oracle.osd_decode_batch(H, pr, s, ps, method, order)
        for b in range(s.shape[0]):
            r0, rw = oracle.osd_decode(H, pr, s[b], ps[b], method, order)
            assert np.array_equal(c0[b], r0) and np.array_equal(cw[b], rw), b


def test_native_osd_matches_c_restatement_n1600_osd_e10(oracle):
    """The native host OSD stage == the C restatement at hgp_34_n1600, OSD-E(10) (the
    notebooks' decoder2 on the headline code), on the oracle's BP posteriors."""
    H = codes.get_code("hgp_34_n1600").hz.astype(np.uint8)
    p = 0.06
    synd, _ = _syndromes(H, p, 48, seed=1600)
    probs = np.full(H.shape[1], p)
    corr, _, conv, post = oracle.bp_decode_batch_soft(H, probs, 160, 0.625, synd)
    nc = np.flatnonzero(~conv)
    assert nc.size >= 8
    o0, ow = HostOSD(H, probs, "osd_e", 10).decode_batch(synd, post, conv, corr, threads=4)
    c0, cw = oracle.osd_decode_batch(H, probs, synd[nc], post[nc], "osd_e", 10)
    assert np.array_equal(o0[nc], c0) and np.array_equal(ow[nc], cw)
