"""ctypes wrapper of the CPU restatement (oracle/qldpc_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py — never by the product package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libqldpc_oracle.so")

_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")


class Counters(ctypes.Structure):
    _fields_ = [("shots", ctypes.c_int64), ("failures", ctypes.c_int64),
                ("sector_decodes", ctypes.c_int64 * 2), ("sector_iters", ctypes.c_int64 * 2),
                ("sector_nonconv", ctypes.c_int64 * 2), ("sector_fail", ctypes.c_int64 * 2)]

    def as_dict(self):
        return {"shots": self.shots, "failures": self.failures,
                "sector_decodes": list(self.sector_decodes), "sector_iters": list(self.sector_iters),
                "sector_nonconv": list(self.sector_nonconv), "sector_fail": list(self.sector_fail)}


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.oracle_bp_decode_batch.restype = ctypes.c_int
        L.oracle_bp_decode_batch.argtypes = [
            ctypes.c_int, ctypes.c_int, _i32p, _i32p, _f64p, ctypes.c_int, ctypes.c_int, ctypes.c_double,
            ctypes.c_int, _u8p, _u8p, _i32p, _u8p, ctypes.c_int64, ctypes.c_int]
        L.oracle_bp_decode_batch_soft.restype = ctypes.c_int
        L.oracle_bp_decode_batch_soft.argtypes = [
            ctypes.c_int, ctypes.c_int, _i32p, _i32p, _f64p, ctypes.c_int, ctypes.c_double,
            ctypes.c_int, _u8p, _u8p, _i32p, _u8p, _f64p, ctypes.c_int64, ctypes.c_int]
        L.oracle_bp_decode_batch_soft_method.restype = ctypes.c_int
        L.oracle_bp_decode_batch_soft_method.argtypes = [
            ctypes.c_int, ctypes.c_int, _i32p, _i32p, _f64p, ctypes.c_int, ctypes.c_int, ctypes.c_double,
            ctypes.c_int, _u8p, _u8p, _i32p, _u8p, _f64p, ctypes.c_int64, ctypes.c_int]
        L.oracle_philox4x32_10.restype = None
        L.oracle_philox4x32_10.argtypes = [ctypes.POINTER(ctypes.c_uint32)] * 3
        L.oracle_uniform.restype = ctypes.c_double
        L.oracle_uniform.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32]
        L.oracle_mc_run.restype = ctypes.c_int
        _lib = L
    return _lib


STREAM_DATA = 0x51D50001
METHODS = {"product_sum": 0, "minimum_sum": 1}


def _csr(H):
    from qldpc_fault_tolerance_amd.codes import CSR

    c = H if isinstance(H, CSR) else CSR.from_dense(H)
    return c.m, c.n, np.ascontiguousarray(c.row_ptr, np.int32), np.ascontiguousarray(c.col_idx, np.int32)


def bp_decode_batch(H, channel_probs, max_iter, bp_method="minimum_sum", ms_scaling_factor=0.625,
                    synd=None, precision=64, nthreads=0):
    m, n, rp, ci = _csr(H)
    synd = np.ascontiguousarray(np.atleast_2d(np.asarray(synd)).astype(np.uint8) & 1)
    B = synd.shape[0]
    assert synd.shape[1] == m
    corr = np.zeros((B, n), np.uint8)
    iters = np.zeros(B, np.int32)
    conv = np.zeros(B, np.uint8)
    probs = np.ascontiguousarray(np.broadcast_to(np.asarray(channel_probs, np.float64), (n,)))
    rc = lib().oracle_bp_decode_batch(m, n, rp, ci, probs, int(max_iter), METHODS[bp_method],
                                      float(ms_scaling_factor), int(precision), synd, corr, iters, conv,
                                      B, int(nthreads))
    if rc:
        raise RuntimeError("oracle_bp_decode_batch failed")
    return corr, iters, conv.astype(bool)


def bp_decode_batch_soft(H, channel_probs, max_iter, ms_scaling_factor=0.625, synd=None, precision=64,
                         nthreads=0, bp_method="minimum_sum"):
    """BP that also returns the final ``log_prob_ratios`` [B, n] (OSD's sort key): min-sum's posterior
    sums, or (``bp_method="product_sum"``) ldpc's ``log(1 / ratio)`` of ``bp_decode_prob_ratios``."""
    m, n, rp, ci = _csr(H)
    synd = np.ascontiguousarray(np.atleast_2d(np.asarray(synd)).astype(np.uint8) & 1)
    B = synd.shape[0]
    assert synd.shape[1] == m
    corr = np.zeros((B, n), np.uint8)
    iters = np.zeros(B, np.int32)
    conv = np.zeros(B, np.uint8)
    post = np.zeros((B, n), np.float64)
    probs = np.ascontiguousarray(np.broadcast_to(np.asarray(channel_probs, np.float64), (n,)))
    rc = lib().oracle_bp_decode_batch_soft_method(m, n, rp, ci, probs, int(max_iter), METHODS[bp_method],
                                                  float(ms_scaling_factor), int(precision), synd, corr, iters, conv,
                                                  post, B, int(nthreads))
    if rc:
        raise RuntimeError("oracle_bp_decode_batch_soft failed")
    return corr, iters, conv.astype(bool), post


OSD_METHODS = {"osd_0": 0, "osd0": 0, "osd_e": 1, "osde": 1, "exhaustive": 1, "osd_cs": 2, "osdcs": 2,
               "combination_sweep": 2}


def _gf2_rank(H):
    A = (np.asarray(H) % 2).astype(np.uint8).copy()
    m, n = A.shape
    r = 0
    for c in range(n):
        piv = np.flatnonzero(A[r:, c])
        if piv.size == 0:
            continue
        p = r + piv[0]
        A[[r, p]] = A[[p, r]]
        below = np.flatnonzero(A[:, c])
        below = below[below != r]
        A[below] ^= A[r]
        r += 1
        if r == m:
            break
    return r


def osd_decode(H, channel_probs, synd, post, osd_method="osd_e", osd_order=10):
    """ldpc 0.1 ``bposd_decoder.osd`` restated literally (pure numpy, small codes only).

    Follows the structure of the reference's OSD dependency (src/Decoders.py:29-36
    builds ``bposd_decoder``; ``decode`` returns ``osdw_decoding``, :39-41):
    stable ascending sort of the columns by ``post`` (log_prob_ratios), Neal's
    ``mod2sparse_decomp`` with the "first" strategy on that order (pivot column
    swapped into position i, pivot row = first remaining row of the partially
    eliminated column), OSD-0 by forward/back substitution on the LU factors,
    then the candidates of ``osd_method`` (osd_e: all 2^w inputs on the first
    w = min(order, n-rank) non-pivot columns in natural binary order; osd_cs:
    weight-1 on every non-pivot column, then weight-2 inside the first w), each
    solved the same way; the first candidate of strictly smaller
    sum_{j: x_j=1} log(1/p_j) wins.  Returns (osd0, osdw) uint8 [n].
    Parity unpinned: ldpc/bposd are absent, so this is the published algorithm,
    not a replay of the package.
    """
    H = (np.asarray(H) % 2).astype(np.uint8)
    m, n = H.shape
    p = np.broadcast_to(np.asarray(channel_probs, np.float64), (n,))
    wts = np.log(1.0 / p)
    s = (np.asarray(synd).astype(np.int64) % 2).astype(np.uint8)
    rank = _gf2_rank(H)
    cols = list(np.argsort(np.asarray(post, np.float64), kind="stable"))
    rows = list(range(m))
    rinv = list(range(m))
    Bm = H.copy()
    ops = []  # (pivot row, rows it was added to)
    for i in range(rank):
        found = None
        for k in range(i, n):
            for r in range(m):
                if Bm[r, cols[k]] and rinv[r] >= i:
                    found = (k, r)
                    break
            if found:
                break
        k, r = found
        cols[k], cols[i] = cols[i], cols[k]
        kr = rinv[r]
        rows[kr], rows[i] = rows[i], rows[kr]
        rinv[rows[kr]] = kr
        rinv[rows[i]] = i
        c = cols[i]
        tgt = [r2 for r2 in range(m) if Bm[r2, c] and rinv[r2] > i]
        for r2 in tgt:
            Bm[r2] ^= Bm[r]
        ops.append((r, tgt))
    piv, ht = cols[:rank], cols[rank:]

    def solve(g):
        g = g.copy()
        for r, tgt in ops:
            if g[r]:
                for r2 in tgt:
                    g[r2] ^= 1
        x = np.zeros(n, np.uint8)
        for i in range(rank - 1, -1, -1):
            acc = g[rows[i]]
            for j in range(i + 1, rank):
                acc ^= Bm[rows[i], piv[j]] & x[piv[j]]
            x[piv[i]] = acc
        return x

    def weight(x):
        t = 0.0
        for j in range(n):
            if x[j]:
                t += wts[j]
        return t

    osd0 = solve(s)
    meth = OSD_METHODS[osd_method] if isinstance(osd_method, str) else int(osd_method)
    k = n - rank
    if meth == 0 or osd_order == 0 or k == 0:
        return osd0, osd0.copy()
    w = min(int(osd_order), k)
    if meth == 1:
        inputs = [[j for j in range(w) if (l >> j) & 1] for l in range(1 << w)]
    else:
        inputs = [[j] for j in range(k)] + [[i, j] for i in range(w) for j in range(w) if j > i]
    best, best_w = osd0.copy(), weight(osd0)
    for t in inputs:
        g = s.copy()
        for j in t:
            g ^= H[:, ht[j]]
        x = solve(g)
        for j in t:
            x[ht[j]] = 1
        wx = weight(x)
        if wx < best_w:
            best, best_w = x, wx
    return osd0, best


def osd_decode_batch(H, channel_probs, synd, post, osd_method="osd_e", osd_order=10, nthreads=0):
    """:func:`osd_decode` restated in C (oracle_osd_decode_batch): the same algorithm step
    for step, fast enough for n1600 OSD-E(10).  Every syndrome is decoded (the caller keeps
    BP's answer where BP converged).  Returns (osd0, osdw) uint8 [B, n]."""
    m, n, rp, ci = _csr(H)
    synd = np.ascontiguousarray(np.atleast_2d(np.asarray(synd)).astype(np.uint8) & 1)
    post = np.ascontiguousarray(np.atleast_2d(np.asarray(post, np.float64)))
    B = synd.shape[0]
    assert synd.shape[1] == m and post.shape == (B, n)
    probs = np.ascontiguousarray(np.broadcast_to(np.asarray(channel_probs, np.float64), (n,)))
    o0 = np.zeros((B, n), np.uint8)
    ow = np.zeros((B, n), np.uint8)
    meth = OSD_METHODS[osd_method] if isinstance(osd_method, str) else int(osd_method)
    L = lib()
    L.oracle_osd_decode_batch.restype = ctypes.c_int
    L.oracle_osd_decode_batch.argtypes = [ctypes.c_int, ctypes.c_int, _i32p, _i32p, _f64p, ctypes.c_int,
                                          ctypes.c_int, _u8p, _f64p, _u8p, _u8p, ctypes.c_int64, ctypes.c_int]
    if L.oracle_osd_decode_batch(m, n, rp, ci, probs, meth, int(osd_order), synd, post, o0, ow, B, int(nthreads)):
        raise RuntimeError("oracle_osd_decode_batch failed")
    return o0, ow


def philox4x32_10(ctr, key):
    c = (ctypes.c_uint32 * 4)(*ctr)
    k = (ctypes.c_uint32 * 2)(*key)
    o = (ctypes.c_uint32 * 4)()
    lib().oracle_philox4x32_10(c, k, o)
    return list(o)


def uniform(seed, shot, qubit, stream=STREAM_DATA):
    return lib().oracle_uniform(seed, shot, qubit, stream)


def mc_run(code, px, py, pz, seed, shot_begin, shot_count, logical_mode="X", max_iter=None,
           bp_method="minimum_sum", ms_scaling_factor=0.625, precision=64, probs_x=None, probs_z=None,
           uniforms=None, per_shot=False, nthreads=0):
    """Fused data-error shot loop on the CPU (oracle / CPU baseline)."""
    n = code.N
    hz, lz, hx, lx = code.csr("hz"), code.csr("lz"), code.csr("hx"), code.csr("lx")
    if probs_x is None:
        probs_x = (px + py)
    if probs_z is None:
        probs_z = (pz + py)
    px_arr = np.ascontiguousarray(np.broadcast_to(np.asarray(probs_x, np.float64), (n,)))
    pz_arr = np.ascontiguousarray(np.broadcast_to(np.asarray(probs_z, np.float64), (n,)))
    if max_iter is None:
        max_iter = int(n / 10)
    mode = {"X": 0, "Z": 1, "Total": 2}[logical_mode]
    S = int(shot_count)
    fail = err = corr = iters = None
    if per_shot:
        fail = np.zeros(S, np.uint8)
        err = np.zeros((S, n), np.uint8)
        corr = np.zeros((S, 2, n), np.uint8)
        iters = np.zeros((S, 2), np.int32)
    if uniforms is not None:
        uniforms = np.ascontiguousarray(uniforms, np.float64)
        assert uniforms.shape == (S, n)
    cnt = Counters()

    def p(a, t):
        return a.ctypes.data_as(ctypes.POINTER(t)) if a is not None else None

    i32 = ctypes.c_int32
    keep = [np.ascontiguousarray(a, np.int32) for a in
            (hz.row_ptr, hz.col_idx, lz.row_ptr, lz.col_idx, hx.row_ptr, hx.col_idx, lx.row_ptr, lx.col_idx)]
    L = lib()
    rc = L.oracle_mc_run(
        ctypes.c_int(n),
        ctypes.c_int(hz.m), p(keep[0], i32), p(keep[1], i32),
        ctypes.c_int(lz.m), p(keep[2], i32), p(keep[3], i32),
        p(px_arr, ctypes.c_double),
        ctypes.c_int(hx.m), p(keep[4], i32), p(keep[5], i32),
        ctypes.c_int(lx.m), p(keep[6], i32), p(keep[7], i32),
        p(pz_arr, ctypes.c_double),
        ctypes.c_int(int(max_iter)), ctypes.c_int(int(max_iter)), ctypes.c_int(METHODS[bp_method]),
        ctypes.c_double(ms_scaling_factor), ctypes.c_int(precision),
        ctypes.c_double(px), ctypes.c_double(py), ctypes.c_double(pz), ctypes.c_uint64(seed),
        ctypes.c_uint64(shot_begin), ctypes.c_int64(S), ctypes.c_int(mode),
        p(uniforms, ctypes.c_double), ctypes.byref(cnt),
        p(fail, ctypes.c_uint8), p(err, ctypes.c_uint8), p(corr, ctypes.c_uint8), p(iters, ctypes.c_int32),
        ctypes.c_int(int(nthreads)))
    del keep
    if rc:
        raise RuntimeError("oracle_mc_run failed")
    out = cnt.as_dict()
    if per_shot:
        out.update(fail=fail, err=err, corr=corr, iters=iters)
    return out


STREAM_PHEN = 0x51D50002


def phenl_trace_len(code, num_rep, num_rounds):
    mx, mz = code.hx.shape[0], code.hz.shape[0]
    return (num_rounds - 1) * num_rep * (mx + mz) + mx + mz


def phenl_run(code, px, py, pz, q, seed, shot_begin, shot_count, num_rounds, num_rep, logical_mode="Total",
              p_data=None, p_synd=None, max_iter_st=None, max_iter_2=None, bp_method="minimum_sum",
              ms_scaling_factor=0.625, precision=64, uniforms=None, per_shot=False, nthreads=0,
              osd_method=None, osd_order=10, firstmin_max_iter=None):
    """Phenomenological space-time shot loop on the CPU (CodeSimulator_Phenon_SpaceTime restated).

    ``osd_method`` (e.g. "osd_e"): decoder2 is BPOSD_Decoder (min-sum BP, then the C OSD
    restatement on the final posteriors when BP did not converge), as the notebooks use.
    ``firstmin_max_iter``: decoder1 is FirstMinBPDecoder (src/Decoders.py:49-74) with that many
    accepted steps at most (min-sum; ``max_iter_st`` unused)."""
    n = code.N
    hz, lz, hx, lx = code.csr("hz"), code.csr("lz"), code.csr("hx"), code.csr("lx")
    mz, mx = hz.m, hx.m
    if p_data is None:
        p_data = px + py
    if p_synd is None:
        p_synd = p_data
    if max_iter_st is None:
        max_iter_st = int(n / 10)
    if max_iter_2 is None:
        max_iter_2 = int(n / 10)
    pst_x = np.ascontiguousarray(np.hstack([p_data * np.ones(n), p_synd * np.ones(mz)] * num_rep))
    pst_z = np.ascontiguousarray(np.hstack([p_data * np.ones(n), p_synd * np.ones(mx)] * num_rep))
    p2 = np.ascontiguousarray(p_data * np.ones(n))
    mode = {"X": 0, "Z": 1, "Total": 2}[logical_mode]
    S = int(shot_count)
    tl = phenl_trace_len(code, num_rep, num_rounds)
    fail = trace = None
    if per_shot:
        fail = np.zeros(S, np.uint8)
        trace = np.zeros((S, tl), np.uint8)
    if uniforms is not None:
        uniforms = np.ascontiguousarray(uniforms, np.float64)
        assert uniforms.shape == (S, ((num_rounds - 1) * num_rep + 1) * (n + mx + mz))
    cnt = Counters()

    def p(a, t):
        return a.ctypes.data_as(ctypes.POINTER(t)) if a is not None else None

    i32, f64 = ctypes.c_int32, ctypes.c_double
    keep = [np.ascontiguousarray(a, np.int32) for a in
            (hz.row_ptr, hz.col_idx, lz.row_ptr, lz.col_idx, hx.row_ptr, hx.col_idx, lx.row_ptr, lx.col_idx)]
    L = lib()
    head = [ctypes.c_int(n),
            ctypes.c_int(mz), p(keep[0], i32), p(keep[1], i32),
            ctypes.c_int(lz.m), p(keep[2], i32), p(keep[3], i32),
            ctypes.c_int(mx), p(keep[4], i32), p(keep[5], i32),
            ctypes.c_int(lx.m), p(keep[6], i32), p(keep[7], i32),
            p(pst_x, f64), p(pst_z, f64), p(p2, f64), p(p2, f64),
            ctypes.c_int(num_rep), ctypes.c_int(int(max_iter_st)), ctypes.c_int(int(max_iter_2))]
    tail = [f64(px), f64(py), f64(pz), f64(q), ctypes.c_uint64(seed), ctypes.c_uint64(shot_begin), ctypes.c_int64(S),
            ctypes.c_int(num_rounds), ctypes.c_int(mode), p(uniforms, f64), ctypes.byref(cnt),
            p(fail, ctypes.c_uint8), p(trace, ctypes.c_uint8), ctypes.c_int(int(nthreads))]
    if firstmin_max_iter is not None:
        assert bp_method == "minimum_sum", "FirstMinBPDecoder: min-sum"
        head[-2] = ctypes.c_int(int(firstmin_max_iter))
        meth = -1 if osd_method is None else (OSD_METHODS[osd_method] if isinstance(osd_method, str) else int(osd_method))
        L.oracle_phenl_run_firstmin.restype = ctypes.c_int
        rc = L.oracle_phenl_run_firstmin(*head, f64(ms_scaling_factor), ctypes.c_int(precision), *tail,
                                         ctypes.c_int(meth), ctypes.c_int(int(osd_order)))
    elif osd_method is None:
        L.oracle_phenl_run.restype = ctypes.c_int
        rc = L.oracle_phenl_run(*head, ctypes.c_int(METHODS[bp_method]), f64(ms_scaling_factor),
                                ctypes.c_int(precision), *tail)
    else:
        assert bp_method == "minimum_sum", "BPOSD_Decoder runs min-sum BP"
        L.oracle_phenl_run_osd.restype = ctypes.c_int
        meth = OSD_METHODS[osd_method] if isinstance(osd_method, str) else int(osd_method)
        rc = L.oracle_phenl_run_osd(*head, f64(ms_scaling_factor), ctypes.c_int(precision), *tail,
                                    ctypes.c_int(meth), ctypes.c_int(int(osd_order)))
    del keep
    if rc:
        raise RuntimeError("oracle_phenl_run failed")
    out = cnt.as_dict()
    if per_shot:
        out.update(fail=fail, trace=trace)
    return out
