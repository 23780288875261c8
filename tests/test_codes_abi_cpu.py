"""CPU tests: code loaders / constructions, the C-ABI library's exports, the distributed helpers."""
import ctypes
import os
import re

import numpy as np
import pytest

from qldpc_fault_tolerance_amd import _native, codes, gf2, parallel

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# [[N, K]] pinned by the reference notebook (.ipynb_checkpoints/Threshold-checkpoint.ipynb:233-236, 263-265, 297-299)
PINNED = {
    "hgp_34_n225": (225, 17), "hgp_34_n625": (625, 25), "hgp_34_n1225_q3": (1225, 49), "hgp_34_n1600": (1600, 64),
    "LP_Matg8_L16_Dmin12": (544, 80), "LP_Matg8_L21_Dmin16": (714, 100), "LP_Matg8_L30_Dmin20": (1020, 136),
    "GenBicycleA1": (126, 12), "GenBicycleA2": (254, 14), "GenBicycleA3": (510, 16),
}


@pytest.mark.parametrize("name,nk", sorted(PINNED.items()))
def test_bundled_code_parameters(name, nk):
    c = codes.get_code(name)
    assert (c.N, c.K) == nk
    assert c.test()
    assert gf2.rank(c.hx) + gf2.rank(c.hz) == c.N - c.K


def test_hgp_formula_rebuilds_n225():
    c = codes.get_code("hgp_34_n225")
    assert c.h1 is not None
    r = codes.hgp(c.h1, c.h2)
    assert np.array_equal(r.hx, c.hx) and np.array_equal(r.hz, c.hz)


def test_synthesized_headline_codes_shape():
    """A14: hgp(h, h) of a (3,4)-regular h; degrees of the Tanner graphs the bench uses."""
    c = codes.get_code("hgp_34_n1600")
    assert c.hx.shape == (768, 1600) and c.hz.shape == (768, 1600)
    assert int(c.hz.sum()) == 5376
    assert set(np.unique(c.hz.sum(0))) == {3, 4} and set(np.unique(c.hz.sum(1))) == {7}


def test_csr_roundtrip_and_matvec():
    rng = np.random.default_rng(0)
    H = (rng.random((30, 50)) < 0.2).astype(np.uint8)
    c = codes.CSR.from_dense(H)
    assert np.array_equal(c.to_dense(), H)
    e = (rng.random((7, 50)) < 0.3).astype(np.uint8)
    assert np.array_equal(c.matvec(e), (e.astype(int) @ H.T.astype(int)) % 2)
    assert np.array_equal(c.matvec(e[0]), (H.astype(int) @ e[0]) % 2)


def test_logicals_anticommute_pairwise():
    c = codes.get_code("GenBicycleA1")
    assert gf2.rank(gf2.matmul(c.lx, c.lz.T)) == c.K
    assert not gf2.matmul(c.hx, c.lz.T).any() and not gf2.matmul(c.hz, c.lx.T).any()


# --------------------------------------------------------------- C ABI


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "qldpc_hip.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*\**(qldpc_\w+)\s*\(", txt, re.M)))


def test_library_exports_every_header_symbol():
    if not os.path.exists(_native.LIB_PATH):
        from qldpc_fault_tolerance_amd.build import build_native

        build_native(verbose=False)
    L = _native.lib()
    syms = _header_symbols()
    assert syms, "no declarations parsed from include/qldpc_hip.h"
    assert sorted(syms) == sorted(_native.EXPORTED)
    for s in syms:
        assert hasattr(L, s), s
    assert L.qldpc_abi_version() == 1


def test_graph_create_validates_on_host():
    L = _native.lib()
    H = codes.CSR.from_dense(np.array([[1, 1, 0], [0, 1, 1]], np.uint8))
    rp = np.ascontiguousarray(H.row_ptr, np.int32)
    ci = np.ascontiguousarray(H.col_idx, np.int32)
    h = ctypes.c_void_p()
    assert L.qldpc_graph_create(0, 2, 3, rp.ctypes.data_as(ctypes.c_void_p), ci.ctypes.data_as(ctypes.c_void_p),
                                ctypes.byref(h)) == 0
    v = [ctypes.c_int32() for _ in range(5)]
    assert L.qldpc_graph_info(h, *[ctypes.byref(x) for x in v]) == 0
    assert [x.value for x in v] == [2, 3, 4, 2, 2]
    L.qldpc_graph_destroy(h)
    bad = np.array([0, 1, 0], np.int32)  # columns not ascending / decreasing row_ptr
    assert L.qldpc_graph_create(0, 2, 3, bad.ctypes.data_as(ctypes.c_void_p), ci.ctypes.data_as(ctypes.c_void_p),
                                ctypes.byref(h)) != 0
    assert b"row_ptr" in L.qldpc_last_error() or b"col_idx" in L.qldpc_last_error()


def test_product_path_fails_loudly_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is visible: the no-GPU failure mode does not apply")
    from qldpc_fault_tolerance_amd.engine import DeviceBP

    c = codes.get_code("hgp_34_n225")
    with pytest.raises((_native.QldpcError, _native.NativeUnavailable)):
        DeviceBP(c.hz, 0.05, max_iter=22)


# ------------------------------------------------------------ sharding


def test_shard_range_partitions_exactly():
    for total in (0, 1, 7, 1000, 1001):
        for ws in (1, 2, 3, 8):
            spans = [parallel.shard_range(total, r, ws, begin=5) for r in range(ws)]
            assert sum(c for _, c in spans) == total
            pos = 5
            for b, c in spans:
                assert b == pos
                pos += c


def _host_graph(L, H):
    csr = codes.CSR.from_dense(np.asarray(H, np.uint8))
    rp = np.ascontiguousarray(csr.row_ptr, np.int32)
    ci = np.ascontiguousarray(csr.col_idx, np.int32)
    h = ctypes.c_void_p()
    assert L.qldpc_graph_create(0, H.shape[0], H.shape[1], rp.ctypes.data_as(ctypes.c_void_p),
                                ci.ctypes.data_as(ctypes.c_void_p), ctypes.byref(h)) == 0
    return h


def test_m2s_annealed_placement_lowers_the_bank_model():
    """qldpc_m2s_place_model runs the decoder build's host half (geometry, degree sort, greedy and
    annealed V-slot placement) and the static LDS model of the m2s variable phase, no device needed.
    On the headline hz graph the default anneal must cut the V-slot read and store conflicts the
    GPU run measured (profiles/r04/passd/model0/1.txt: reads 382 -> 360, stores 676 -> 500), leave
    the CS gathers alone (placement inside rows does not move a check's CS entry), and be
    deterministic (seeded, and memoised per process)."""
    L = _native.lib()
    h = _host_graph(L, codes.get_code("hgp_34_n1600").hz)
    out = (ctypes.c_int64 * 6)()
    try:
        assert L.qldpc_m2s_place_model(h, 0, out) == 0
        greedy = list(out)
        assert L.qldpc_m2s_place_model(h, 2_000_000, out) == 0
        short = list(out)
        assert L.qldpc_m2s_place_model(h, 2_000_000, out) == 0
        assert list(out) == short  # deterministic
    finally:
        L.qldpc_graph_destroy(h)
    assert greedy == [244, 52, 382, 190, 676, 292]  # == the decoder's own model on the GPU box
    assert short[:2] == greedy[:2]
    assert short[3] < greedy[3] and short[5] < greedy[5] - 40
    # every group at least 1 cycle: cost = groups + extra
    assert short[2] - short[3] == greedy[2] - greedy[3] and short[4] - short[5] == greedy[4] - greedy[5]


def test_m2s_place_model_rejects_graphs_outside_the_family():
    L = _native.lib()
    h = _host_graph(L, codes.get_code("LP_Matg8_L30_Dmin20").hz)  # rows of 8, column degree 5
    out = (ctypes.c_int64 * 6)()
    try:
        assert L.qldpc_m2s_place_model(h, 0, out) != 0
        assert b"m2s" in L.qldpc_last_error()
    finally:
        L.qldpc_graph_destroy(h)
