"""Device-side objects of the engine: Tanner graphs, BP decoders, fused MC runs.

Thin owners of the C-ABI handles in ``libqldpc_hip.so``.  PyTorch-ROCm is used
only for device buffers and the current HIP stream; every computation runs in
the hand-written kernels.  No CPU fallback exists (``_native`` raises).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

from . import _native
from .codes import CSR, CSSCode

METHODS = {"product_sum": 0, "prod_sum": 0, "ps": 0, "minimum_sum": 1, "min_sum": 1, "ms": 1}
LOGICAL_MODES = {"X": 0, "Z": 1, "Total": 2}


def _torch():
    import torch

    if not torch.cuda.is_available():
        raise _native.NativeUnavailable("torch reports no HIP device; the engine needs an MI355X (no CPU fallback)")
    return torch


def _stream_handle(torch, device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def bp_method_code(bp_method) -> int:
    if isinstance(bp_method, (int, np.integer)):
        return int(bp_method)
    key = str(bp_method).lower()
    if key not in METHODS:
        raise ValueError(f"unknown bp_method {bp_method!r}")
    return METHODS[key]


class DeviceGraph:
    """A parity-check matrix uploaded once (``qldpc_graph_create``)."""

    def __init__(self, H, device: int | None = None):
        c = H if isinstance(H, CSR) else CSR.from_dense(H)
        if device is None:  # this rank's GPU (LOCAL_RANK under torch.distributed.run)
            from .parallel import local_device_index

            device = local_device_index()
        self.csr = c
        self.m, self.n = c.m, c.n
        self.device = device
        L = _native.lib()
        self._rp = np.ascontiguousarray(c.row_ptr, dtype=np.int32)
        self._ci = np.ascontiguousarray(c.col_idx, dtype=np.int32)
        h = ctypes.c_void_p()
        _native.check(L.qldpc_graph_create(device, c.m, c.n, self._rp.ctypes.data_as(ctypes.c_void_p),
                                           self._ci.ctypes.data_as(ctypes.c_void_p), ctypes.byref(h)),
                      "qldpc_graph_create")
        self.handle = h

    def info(self):
        v = [ctypes.c_int32() for _ in range(5)]
        _native.check(_native.lib().qldpc_graph_info(self.handle, *[ctypes.byref(x) for x in v]), "graph_info")
        return dict(zip(["m", "n", "nnz", "max_row_deg", "max_col_deg"], [x.value for x in v]))

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and _native._lib is not None:
            _native.lib().qldpc_graph_destroy(h)
            self.handle = None


class DeviceBP:
    """``ldpc.bp_decoder`` equivalent on the GPU (``qldpc_bp_create``).

    ``anneal_iters``: moves of the annealed V-slot placement the fp64 engine-3 families run at
    creation (host time, one core: ~0.18 us per move; default 4000 per edge capped at 2^25, memoised
    per process for the same graph).  0 keeps the greedy placement (decodes identically; the placement
    only moves LDS bank conflicts), for short runs over many codes."""

    def __init__(self, H, channel_probs, max_iter: int = 0, bp_method="minimum_sum", ms_scaling_factor=0.625,
                 precision: int = 64, vars_per_thread: int = 0, device: int | None = None, graph: DeviceGraph | None = None,
                 min_col_slots: int = 0, soft: bool = False, hbm: bool = False, anneal_iters: int | None = None):
        if anneal_iters is not None:  # read by qldpc_bp_create (QLDPC_M2S_ANNEAL) at creation only
            old = os.environ.get("QLDPC_M2S_ANNEAL")
            os.environ["QLDPC_M2S_ANNEAL"] = str(int(anneal_iters))
            try:
                self.__init__(H, channel_probs, max_iter, bp_method, ms_scaling_factor, precision, vars_per_thread,
                              device, graph, min_col_slots, soft, hbm, None)
            finally:
                if old is None:
                    os.environ.pop("QLDPC_M2S_ANNEAL", None)
                else:
                    os.environ["QLDPC_M2S_ANNEAL"] = old
            return
        self.graph = graph if graph is not None else DeviceGraph(H, device=device)
        n = self.graph.n
        probs = np.asarray(channel_probs, dtype=np.float64)
        if probs.ndim == 0:
            probs = np.full(n, float(probs))
        if probs.shape != (n,):
            raise ValueError(f"channel_probs must have length {n}")
        self.channel_probs = np.ascontiguousarray(probs)
        self.max_iter = int(max_iter) if int(max_iter) > 0 else n
        self.bp_method = bp_method_code(bp_method)
        self.ms_scaling_factor = float(ms_scaling_factor)
        self.precision = int(precision)
        self.soft = bool(soft)
        h = ctypes.c_void_p()
        if hbm:
            # engine 6: HBM-resident messages (automatic when no LDS engine holds the image)
            if self.bp_method != 1:
                raise NotImplementedError("the HBM-resident engine implements minimum_sum")
            _native.check(_native.lib().qldpc_bp_create_hbm(
                self.graph.handle, self.channel_probs.ctypes.data_as(ctypes.c_void_p), self.max_iter,
                self.ms_scaling_factor, self.precision, ctypes.byref(h)), "qldpc_bp_create_hbm")
        elif self.soft and self.bp_method == 1:
            # BP+OSD: engine 1 hands back the final posteriors (qldpc_bp_create_soft); a product-sum
            # decoder (engine 5) writes ldpc's log(1 / ratio) posteriors from the default create
            _native.check(_native.lib().qldpc_bp_create_soft(
                self.graph.handle, self.channel_probs.ctypes.data_as(ctypes.c_void_p), self.max_iter,
                self.ms_scaling_factor, self.precision, ctypes.byref(h)), "qldpc_bp_create_soft")
        else:
            _native.check(_native.lib().qldpc_bp_create(
                self.graph.handle, self.channel_probs.ctypes.data_as(ctypes.c_void_p), self.max_iter,
                self.bp_method, self.ms_scaling_factor, self.precision, int(vars_per_thread), int(min_col_slots),
                ctypes.byref(h)), "qldpc_bp_create")
        self.handle = h

    @property
    def m(self):
        return self.graph.m

    @property
    def n(self):
        return self.graph.n

    def geometry(self):
        v = [ctypes.c_int32() for _ in range(4)]
        _native.check(_native.lib().qldpc_bp_geometry(self.handle, *[ctypes.byref(x) for x in v]), "bp_geometry")
        e = ctypes.c_int32()
        _native.check(_native.lib().qldpc_bp_engine(self.handle, ctypes.byref(e)), "bp_engine")
        g = dict(zip(["threads", "vars_per_thread", "lds_bytes", "blocks_per_cu"], [x.value for x in v]))
        g["engine"] = e.value
        d = ctypes.c_int32()
        _native.check(_native.lib().qldpc_bp_degree3_slots(self.handle, ctypes.byref(d)), "bp_degree3_slots")
        g["degree3_slots"] = d.value
        b0, b1 = ctypes.c_int32(), ctypes.c_int32()
        _native.check(_native.lib().qldpc_bp_bank_stats(self.handle, ctypes.byref(b0), ctypes.byref(b1)),
                      "bp_bank_stats")
        g["gather_conflicts"] = (b0.value, b1.value)
        kid, nch = ctypes.c_int32(), ctypes.c_int32()
        _native.check(_native.lib().qldpc_bp_kernel_id(self.handle, ctypes.byref(kid), ctypes.byref(nch)),
                      "bp_kernel_id")
        g["kernel_id"], g["row_chunks"] = kid.value, nch.value
        lm = (ctypes.c_int64 * 6)()
        _native.check(_native.lib().qldpc_bp_lds_model(self.handle, lm), "bp_lds_model")
        g["lds_model"] = dict(zip(["cs_gather", "cs_gather_extra", "v_read", "v_read_extra", "v_store", "v_store_extra"],
                                  list(lm)))
        return g

    def decode_batch_device(self, synd_dev, corr_dev, iters_dev=None, conv_dev=None, stream=None):
        """Decode device uint8 syndromes [B, m] into device corrections [B, n] (async)."""
        torch = _torch()
        B = int(synd_dev.shape[0])
        assert synd_dev.dtype == torch.uint8 and synd_dev.is_contiguous() and synd_dev.shape[1] == self.m
        assert corr_dev.dtype == torch.uint8 and corr_dev.is_contiguous() and tuple(corr_dev.shape) == (B, self.n)
        s = stream if stream is not None else _stream_handle(torch, synd_dev.device)
        _native.check(_native.lib().qldpc_bp_decode_batch(
            self.handle, ctypes.c_void_p(synd_dev.data_ptr()), ctypes.c_void_p(corr_dev.data_ptr()),
            ctypes.c_void_p(iters_dev.data_ptr()) if iters_dev is not None else None,
            ctypes.c_void_p(conv_dev.data_ptr()) if conv_dev is not None else None, B, s), "qldpc_bp_decode_batch")

    def decode_batch(self, synd):
        """Host convenience: ``synd`` [B, m] (0/1) -> (corr [B, n] int, iters [B], converged [B])."""
        torch = _torch()
        s = np.ascontiguousarray(np.atleast_2d(np.asarray(synd)).astype(np.int64) % 2, dtype=np.uint8)
        if s.shape[1] != self.m:
            raise ValueError(f"syndrome length {s.shape[1]} != number of checks {self.m}")
        dev = torch.device("cuda", self.graph.device)
        sd = torch.from_numpy(s).to(dev)
        corr = torch.empty((s.shape[0], self.n), dtype=torch.uint8, device=dev)
        iters = torch.empty(s.shape[0], dtype=torch.int32, device=dev)
        conv = torch.empty(s.shape[0], dtype=torch.uint8, device=dev)
        self.decode_batch_device(sd, corr, iters, conv)
        torch.cuda.synchronize(dev)
        return corr.cpu().numpy().astype(np.int64), iters.cpu().numpy(), conv.cpu().numpy().astype(bool)

    def decode_batch_soft(self, synd):
        """Like :meth:`decode_batch` plus the final posteriors ``post`` [B, n] float64
        (ldpc's ``log_prob_ratios``); needs ``soft=True``."""
        torch = _torch()
        s = np.ascontiguousarray(np.atleast_2d(np.asarray(synd)).astype(np.int64) % 2, dtype=np.uint8)
        if s.shape[1] != self.m:
            raise ValueError(f"syndrome length {s.shape[1]} != number of checks {self.m}")
        B = s.shape[0]
        dev = torch.device("cuda", self.graph.device)
        sd = torch.from_numpy(s).to(dev)
        corr = torch.empty((B, self.n), dtype=torch.uint8, device=dev)
        iters = torch.empty(B, dtype=torch.int32, device=dev)
        conv = torch.empty(B, dtype=torch.uint8, device=dev)
        post = torch.empty((B, self.n), dtype=torch.float64, device=dev)
        _native.check(_native.lib().qldpc_bp_decode_batch_soft(
            self.handle, ctypes.c_void_p(sd.data_ptr()), ctypes.c_void_p(corr.data_ptr()),
            ctypes.c_void_p(iters.data_ptr()), ctypes.c_void_p(conv.data_ptr()), ctypes.c_void_p(post.data_ptr()),
            B, _stream_handle(torch, dev)), "qldpc_bp_decode_batch_soft")
        torch.cuda.synchronize(dev)
        return (corr.cpu().numpy().astype(np.int64), iters.cpu().numpy(), conv.cpu().numpy().astype(bool),
                post.cpu().numpy())

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and _native._lib is not None:
            _native.lib().qldpc_bp_destroy(h)
            self.handle = None


OSD_METHODS = {"osd_0": 0, "osd0": 0, "osd_e": 1, "osde": 1, "exhaustive": 1, "osd_cs": 2, "osdcs": 2,
               "combination_sweep": 2}


class HostOSD:
    """Ordered-statistics post-processing stage (``qldpc_osd_*``, csrc/osd.hip).

    Native host code (GF(2) elimination on bit-packed columns, a std::thread
    pool over syndromes); it consumes the GPU BP's posteriors.  Needs only the
    library, not a GPU.
    """

    def __init__(self, H, channel_probs, osd_method="osd_e", osd_order=10):
        c = H if isinstance(H, CSR) else CSR.from_dense(H)
        self.m, self.n = c.m, c.n
        key = str(osd_method).lower() if not isinstance(osd_method, (int, np.integer)) else None
        if key is not None and key not in OSD_METHODS:
            raise ValueError(f"unknown osd_method {osd_method!r}")
        self.osd_method = OSD_METHODS[key] if key is not None else int(osd_method)
        self.osd_order = int(osd_order)
        probs = np.asarray(channel_probs, dtype=np.float64)
        if probs.ndim == 0:
            probs = np.full(self.n, float(probs))
        self._probs = np.ascontiguousarray(probs)
        rp = np.ascontiguousarray(c.row_ptr, dtype=np.int32)
        ci = np.ascontiguousarray(c.col_idx, dtype=np.int32)
        h = ctypes.c_void_p()
        _native.check(_native.lib().qldpc_osd_create(
            self.m, self.n, rp.ctypes.data_as(ctypes.c_void_p), ci.ctypes.data_as(ctypes.c_void_p),
            self._probs.ctypes.data_as(ctypes.c_void_p), self.osd_method, self.osd_order, ctypes.byref(h)),
            "qldpc_osd_create")
        self.handle = h
        r = ctypes.c_int32()
        _native.check(_native.lib().qldpc_osd_rank(h, ctypes.byref(r)), "qldpc_osd_rank")
        self.rank = r.value

    def decode_batch(self, synd, post, conv=None, bp_corr=None, threads: int = 0):
        """(osd0 [B, n], osdw [B, n]) uint8; converged rows (``conv``) copy ``bp_corr``."""
        s = np.ascontiguousarray(np.atleast_2d(np.asarray(synd)).astype(np.int64) % 2, dtype=np.uint8)
        B = s.shape[0]
        pst = np.ascontiguousarray(np.asarray(post, dtype=np.float64).reshape(B, self.n))
        if s.shape[1] != self.m:
            raise ValueError(f"syndrome length {s.shape[1]} != number of checks {self.m}")
        cv = None if conv is None else np.ascontiguousarray(np.asarray(conv).reshape(B), dtype=np.uint8)
        bc = None if bp_corr is None else np.ascontiguousarray(np.asarray(bp_corr).reshape(B, self.n),
                                                                 dtype=np.uint8)
        o0 = np.zeros((B, self.n), np.uint8)
        ow = np.zeros((B, self.n), np.uint8)
        vp = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        _native.check(_native.lib().qldpc_osd_decode_batch(self.handle, vp(s), vp(pst), vp(cv), vp(bc), vp(o0),
                                                           vp(ow), B, int(threads)), "qldpc_osd_decode_batch")
        return o0, ow

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and _native._lib is not None:
            _native.lib().qldpc_osd_destroy(h)
            self.handle = None


class DeviceOSD:
    """OSD on the GPU (``qldpc_osd_gpu_*``): one workgroup per non-converged syndrome, fed
    straight from the soft-output BP's device buffers.  Uniform priors weigh candidates by
    popcount; non-uniform ones (the circuit-level DEM priors) by sum log(1/p_j) in column order,
    as the host stage.  ``supported`` says whether a graph qualifies (n <= 8192, osd_e order <= 24)."""

    MAX_N = 8192

    @staticmethod
    def supported(n, channel_probs, osd_method, osd_order) -> bool:
        p = np.broadcast_to(np.asarray(channel_probs, dtype=np.float64), (n,))
        key = str(osd_method).lower() if not isinstance(osd_method, (int, np.integer)) else None
        meth = OSD_METHODS.get(key, -1) if key is not None else int(osd_method)
        return (n <= DeviceOSD.MAX_N and bool(np.all((p > 0) & (p < 1))) and meth in (0, 1, 2)
                and not (meth == 1 and int(osd_order) > 24))

    def __init__(self, graph: DeviceGraph, channel_probs, osd_method="osd_e", osd_order=10):
        self.graph = graph
        n = graph.n
        key = str(osd_method).lower() if not isinstance(osd_method, (int, np.integer)) else None
        if key is not None and key not in OSD_METHODS:
            raise ValueError(f"unknown osd_method {osd_method!r}")
        self.osd_method = OSD_METHODS[key] if key is not None else int(osd_method)
        self.osd_order = int(osd_order)
        probs = np.asarray(channel_probs, dtype=np.float64)
        self._probs = np.ascontiguousarray(np.full(n, float(probs)) if probs.ndim == 0 else probs)
        h = ctypes.c_void_p()
        _native.check(_native.lib().qldpc_osd_gpu_create(graph.handle, self._probs.ctypes.data_as(ctypes.c_void_p),
                                                         self.osd_method, self.osd_order, ctypes.byref(h)),
                      "qldpc_osd_gpu_create")
        self.handle = h

    def geometry(self) -> dict:
        """The elimination layout the handle chose: register-row words, column-window words (0 =
        none), threads per workgroup and the persistent grid."""
        v = [ctypes.c_int32() for _ in range(4)]
        _native.check(_native.lib().qldpc_osd_gpu_geometry(self.handle, *[ctypes.byref(x) for x in v]),
                      "qldpc_osd_gpu_geometry")
        return dict(zip(("row_words", "window_words", "threads", "workgroups"), (x.value for x in v)))

    def decode_device(self, synd_dev, post_dev, conv_dev, corr_dev, out0_dev, outw_dev, stream=None):
        torch = _torch()
        B = int(synd_dev.shape[0])
        s = stream if stream is not None else _stream_handle(torch, synd_dev.device)

        def ptr(t):
            return ctypes.c_void_p(t.data_ptr()) if t is not None else None

        _native.check(_native.lib().qldpc_osd_gpu_decode(self.handle, ptr(synd_dev), ptr(post_dev), ptr(conv_dev),
                                                         ptr(corr_dev), ptr(out0_dev), ptr(outw_dev), B, s),
                      "qldpc_osd_gpu_decode")

    def bposd_batch(self, bp: "DeviceBP", synd, host_post: bool = True):
        """Soft BP (``bp``, soft=True) then GPU OSD, all on the device: ``synd`` [B, m] ->
        (osdw, osd0, bp_corr, iters, conv, post) as host arrays (``post`` stays a device
        tensor when ``host_post`` is False: 8 bytes per variable not worth copying back)."""
        torch = _torch()
        s = np.ascontiguousarray(np.atleast_2d(np.asarray(synd)).astype(np.int64) % 2, dtype=np.uint8)
        B, n = s.shape[0], self.graph.n
        dev = torch.device("cuda", self.graph.device)
        sd = torch.from_numpy(s).to(dev)
        corr = torch.empty((B, n), dtype=torch.uint8, device=dev)
        iters = torch.empty(B, dtype=torch.int32, device=dev)
        conv = torch.empty(B, dtype=torch.uint8, device=dev)
        post = torch.empty((B, n), dtype=torch.float64, device=dev)
        o0 = torch.empty((B, n), dtype=torch.uint8, device=dev)
        ow = torch.empty((B, n), dtype=torch.uint8, device=dev)
        st = _stream_handle(torch, dev)
        _native.check(_native.lib().qldpc_bp_decode_batch_soft(
            bp.handle, ctypes.c_void_p(sd.data_ptr()), ctypes.c_void_p(corr.data_ptr()),
            ctypes.c_void_p(iters.data_ptr()), ctypes.c_void_p(conv.data_ptr()), ctypes.c_void_p(post.data_ptr()),
            B, st), "qldpc_bp_decode_batch_soft")
        self.decode_device(sd, post, conv, corr, o0, ow, st)
        torch.cuda.synchronize(dev)
        return (ow.cpu().numpy(), o0.cpu().numpy(), corr.cpu().numpy().astype(np.int64), iters.cpu().numpy(),
                conv.cpu().numpy().astype(bool), post.cpu().numpy() if host_post else post)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and _native._lib is not None:
            _native.lib().qldpc_osd_gpu_destroy(h)
            self.handle = None


class DeviceFirstMin:
    """``FirstMinBPDecoder`` (``src/Decoders.py:49-74``) on the GPU (``qldpc_firstmin_*``): one-iteration
    min-sum BP repeated on the running syndrome while its weight does not grow, at most
    ``max_iter`` accepted steps, the whole loop in one kernel (one workgroup per syndrome)."""

    def __init__(self, H, channel_probs, max_iter: int, ms_scaling_factor=0.625, precision: int = 64,
                 device: int | None = None, graph: DeviceGraph | None = None):
        self.graph = graph if graph is not None else DeviceGraph(H, device=device)
        n = self.graph.n
        probs = np.asarray(channel_probs, dtype=np.float64)
        self._probs = np.ascontiguousarray(np.full(n, float(probs)) if probs.ndim == 0 else probs)
        if self._probs.shape != (n,):
            raise ValueError(f"channel_probs must have {n} entries")
        self.max_iter = int(max_iter)
        h = ctypes.c_void_p()
        _native.check(_native.lib().qldpc_firstmin_create(self.graph.handle, self._probs.ctypes.data_as(ctypes.c_void_p),
                                                          self.max_iter, float(ms_scaling_factor), int(precision),
                                                          ctypes.byref(h)), "qldpc_firstmin_create")
        self.handle = h

    def decode_device(self, synd_dev, corr_dev, steps_dev=None, stream=None):
        torch = _torch()
        s = stream if stream is not None else _stream_handle(torch, synd_dev.device)
        _native.check(_native.lib().qldpc_firstmin_decode(
            self.handle, ctypes.c_void_p(synd_dev.data_ptr()), ctypes.c_void_p(corr_dev.data_ptr()),
            ctypes.c_void_p(steps_dev.data_ptr()) if steps_dev is not None else None, int(synd_dev.shape[0]), s),
            "qldpc_firstmin_decode")

    def decode_batch(self, synd):
        """[B, m] syndromes -> (corrections [B, n] int64, accepted steps [B] int32)."""
        torch = _torch()
        S = np.ascontiguousarray(np.atleast_2d(np.asarray(synd)).astype(np.int64) % 2, dtype=np.uint8)
        B, n = S.shape[0], self.graph.n
        if S.shape[1] != self.graph.m:
            raise ValueError(f"syndromes must have {self.graph.m} columns")
        dev = torch.device("cuda", self.graph.device)
        sd = torch.from_numpy(S).to(dev)
        corr = torch.empty((B, n), dtype=torch.uint8, device=dev)
        steps = torch.empty(B, dtype=torch.int32, device=dev)
        self.decode_device(sd, corr, steps)
        torch.cuda.synchronize(dev)
        return corr.cpu().numpy().astype(np.int64), steps.cpu().numpy()

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and _native._lib is not None:
            _native.lib().qldpc_firstmin_destroy(h)
            self.handle = None


@dataclass
class MCResult:
    shots: int
    failures: int
    sector_decodes: list
    sector_iters: list
    sector_nonconv: list
    sector_fail: list
    iter_hist: np.ndarray  # [2, HIST_BINS]
    fail: np.ndarray | None = None
    err: np.ndarray | None = None
    corr: np.ndarray | None = None
    iters: np.ndarray | None = None
    trace: np.ndarray | None = None
    detobs: np.ndarray | None = None

    @staticmethod
    def from_words(w: np.ndarray) -> "MCResult":
        w = np.asarray(w, dtype=np.int64)
        hb = _native.HIST_BINS
        return MCResult(int(w[0]), int(w[1]), w[2:4].tolist(), w[4:6].tolist(), w[6:8].tolist(), w[8:10].tolist(),
                        w[10:10 + 2 * hb].reshape(2, hb).copy())

    def merge(self, o: "MCResult") -> "MCResult":
        return MCResult(self.shots + o.shots, self.failures + o.failures,
                        [a + b for a, b in zip(self.sector_decodes, o.sector_decodes)],
                        [a + b for a, b in zip(self.sector_iters, o.sector_iters)],
                        [a + b for a, b in zip(self.sector_nonconv, o.sector_nonconv)],
                        [a + b for a, b in zip(self.sector_fail, o.sector_fail)], self.iter_hist + o.iter_hist)


class DeviceMC:
    """Fused shot loop of ``CodeSimulator_DataError`` on one GPU (``qldpc_mc_*``).

    Sector X decodes X errors with the hz decoder and checks lz; sector Z
    decodes Z errors with the hx decoder and checks lx.
    """

    def __init__(self, code: CSSCode, dec_x: DeviceBP | None, dec_z: DeviceBP | None):
        self.code = code
        self.dec_x, self.dec_z = dec_x, dec_z
        dev = (dec_x or dec_z).graph.device
        self.device = dev
        self.lz = DeviceGraph(code.csr("lz"), device=dev) if dec_x is not None else None
        self.lx = DeviceGraph(code.csr("lx"), device=dev) if dec_z is not None else None
        h = ctypes.c_void_p()
        _native.check(_native.lib().qldpc_mc_create(
            dec_x.handle if dec_x else None, self.lz.handle if self.lz else None,
            dec_z.handle if dec_z else None, self.lx.handle if self.lx else None, ctypes.byref(h)),
            "qldpc_mc_create")
        self.handle = h

    def set_osd(self, osd_x: "DeviceOSD | None", osd_z: "DeviceOSD | None"):
        """BP+OSD in the fused loop (``qldpc_mc_set_osd``): decodes that reach max_iter go through the
        GPU OSD stage and their failures are re-checked on the device."""
        self._osd = (osd_x, osd_z)  # keep the handles alive
        _native.check(_native.lib().qldpc_mc_set_osd(self.handle, osd_x.handle if osd_x is not None else None,
                                                     osd_z.handle if osd_z is not None else None), "qldpc_mc_set_osd")

    def new_counters(self):
        torch = _torch()
        return torch.zeros(_native.COUNTER_WORDS, dtype=torch.int64, device=torch.device("cuda", self.device))

    def launch(self, px, py, pz, seed, shot_begin, shot_count, logical_mode="X", counters=None, uniforms=None,
               fail=None, err=None, corr=None, iters=None, grid_blocks=0, stream=None):
        """Asynchronous launch on the current stream; counters accumulate in ``counters`` (device int64)."""
        torch = _torch()
        if counters is None:
            raise ValueError("counters buffer required")
        mode = LOGICAL_MODES[logical_mode] if isinstance(logical_mode, str) else int(logical_mode)
        s = stream if stream is not None else _stream_handle(torch, counters.device)

        def ptr(t):
            return ctypes.c_void_p(t.data_ptr()) if t is not None else None

        _native.check(_native.lib().qldpc_mc_launch(
            self.handle, float(px), float(py), float(pz), int(seed) & (2**64 - 1), int(shot_begin), int(shot_count),
            mode, ptr(uniforms), ptr(counters), ptr(fail), ptr(err), ptr(corr), ptr(iters), int(grid_blocks), s),
            "qldpc_mc_launch")

    def run(self, px, py, pz, seed, shot_begin, shot_count, logical_mode="X", uniforms=None, per_shot=False,
            grid_blocks=0) -> MCResult:
        torch = _torch()
        dev = torch.device("cuda", self.device)
        n = self.code.N
        S = int(shot_count)
        cnt = self.new_counters()
        u = torch.from_numpy(np.ascontiguousarray(uniforms, dtype=np.float64)).to(dev) if uniforms is not None else None
        if u is not None and tuple(u.shape) != (S, n):
            raise ValueError(f"uniforms must be [{S}, {n}]")
        f = e = c = it = None
        if per_shot:
            f = torch.zeros(S, dtype=torch.uint8, device=dev)
            e = torch.zeros((S, n), dtype=torch.uint8, device=dev)
            c = torch.zeros((S, 2, n), dtype=torch.uint8, device=dev)
            it = torch.zeros((S, 2), dtype=torch.int32, device=dev)
        self.launch(px, py, pz, seed, shot_begin, S, logical_mode, cnt, u, f, e, c, it, grid_blocks)
        torch.cuda.synchronize(dev)
        res = MCResult.from_words(cnt.cpu().numpy())
        if per_shot:
            res.fail, res.err, res.corr, res.iters = f.cpu().numpy(), e.cpu().numpy(), c.cpu().numpy(), it.cpu().numpy()
        return res

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and _native._lib is not None:
            _native.lib().qldpc_mc_destroy(h)
            self.handle = None


def sample_errors(n, px, py, pz, seed, shot_begin, shot_count, uniforms=None, device: int | None = None,
                  stream=None):
    """``qldpc_sample_errors``: the sampling step of the fused kernels alone
    (``CodeSimulator_DataError._generate_error``, src/Simulators.py:89-115) as a uint8
    ``[S, n]`` device tensor (bit0 = x, bit1 = z), from the Philox stream keyed by the
    global shot index or from external uniforms ``[S, n]`` (CPython ``random()`` values)."""
    torch = _torch()
    if device is None:
        from .parallel import local_device_index

        device = local_device_index()
    dev = torch.device("cuda", device)
    S = int(shot_count)
    out = torch.empty((S, int(n)), dtype=torch.uint8, device=dev)
    u = None
    if uniforms is not None:
        u = uniforms if isinstance(uniforms, torch.Tensor) else torch.from_numpy(
            np.ascontiguousarray(uniforms, dtype=np.float64))
        u = u.to(dev, dtype=torch.float64).contiguous()
        if tuple(u.shape) != (S, int(n)):
            raise ValueError(f"uniforms must be [{S}, {n}]")
    s = stream if stream is not None else _stream_handle(torch, dev)
    with torch.cuda.device(dev):
        _native.check(_native.lib().qldpc_sample_errors(
            float(px), float(py), float(pz), int(seed) & (2**64 - 1), int(shot_begin), S, int(n),
            ctypes.c_void_p(u.data_ptr()) if u is not None else None, ctypes.c_void_p(out.data_ptr()), s),
            "qldpc_sample_errors")
    return out


def run_sharded(mcs, comms, px, py, pz, seed, shot_begin, shot_count, logical_mode="Total") -> MCResult:
    """``qldpc_mc_run_sharded``: one host thread drives one :class:`DeviceMC` per GPU (each on its
    own device's decoders) over contiguous blocks of the global shots, and sums the counters with
    one grouped RCCL all-reduce (``comms`` from :meth:`parallel.NativeComm.init_all`, same device
    order; None for one device).  The totals equal one device running all the shots."""
    mcs = list(mcs)
    nd = len(mcs)
    arr = (ctypes.c_void_p * nd)(*[m.handle.value for m in mcs])
    carr = None
    if comms is not None:
        comms = list(comms)
        if len(comms) != nd:
            raise ValueError("one communicator per MC handle")
        carr = (ctypes.c_void_p * nd)(*[c.handle.value for c in comms])
    out = _native.Counters()
    mode = LOGICAL_MODES[logical_mode] if isinstance(logical_mode, str) else int(logical_mode)
    _native.check(_native.lib().qldpc_mc_run_sharded(
        ctypes.cast(arr, ctypes.POINTER(ctypes.c_void_p)),
        ctypes.cast(carr, ctypes.POINTER(ctypes.c_void_p)) if carr is not None else None, nd, float(px), float(py),
        float(pz), int(seed) & (2**64 - 1), int(shot_begin), int(shot_count), mode, ctypes.byref(out)),
        "qldpc_mc_run_sharded")
    return MCResult.from_words(np.frombuffer(bytes(out), dtype=np.int64))


class DevicePhenl:
    """Phenomenological space-time shot loop of ``CodeSimulator_Phenon_SpaceTime`` on one GPU (``qldpc_phenl_*``).

    ``st_x`` / ``st_z`` decode the X / Z detector histories on the space-time
    graphs of hz / hx; ``dec2_x`` / ``dec2_z`` decode the perfect final round.
    """

    def __init__(self, code: CSSCode, st_x: DeviceBP, st_z: DeviceBP, dec2_x: DeviceBP, dec2_z: DeviceBP,
                 num_rep: int, max_batch: int = 0):
        self.code = code
        self.num_rep = int(num_rep)
        self.decoders = (st_x, st_z, dec2_x, dec2_z)
        dev = dec2_x.graph.device
        self.device = dev
        self.lz = DeviceGraph(code.csr("lz"), device=dev)
        self.lx = DeviceGraph(code.csr("lx"), device=dev)
        h = ctypes.c_void_p()
        _native.check(_native.lib().qldpc_phenl_create(
            st_x.handle, st_z.handle, dec2_x.handle, dec2_z.handle, self.lz.handle, self.lx.handle, self.num_rep,
            int(max_batch), ctypes.byref(h)), "qldpc_phenl_create")
        self.handle = h

    def set_final_osd(self, osd_x: "DeviceOSD | None", osd_z: "DeviceOSD | None"):
        """BP+OSD final round (decoder2 = BPOSD_Decoder): ``qldpc_phenl_set_final_osd``."""
        for o, d in ((osd_x, self.decoders[2]), (osd_z, self.decoders[3])):
            if o is not None and o.graph.n != d.n:
                raise ValueError("OSD graph does not match the final-round decoder")
        self._osd2 = (osd_x, osd_z)  # keep the handles alive
        _native.check(_native.lib().qldpc_phenl_set_final_osd(
            self.handle, osd_x.handle if osd_x is not None else None, osd_z.handle if osd_z is not None else None),
            "qldpc_phenl_set_final_osd")

    def set_round_firstmin(self, fm_x: "DeviceFirstMin | None", fm_z: "DeviceFirstMin | None"):
        """Noisy rounds decoded by FirstMinBPDecoder (``qldpc_phenl_set_round_firstmin``): each
        handle must be built on exactly its sector's space-time graph."""
        self._fm1 = (fm_x, fm_z)  # keep the handles alive
        _native.check(_native.lib().qldpc_phenl_set_round_firstmin(
            self.handle, fm_x.handle if fm_x is not None else None, fm_z.handle if fm_z is not None else None),
            "qldpc_phenl_set_round_firstmin")

    def trace_len(self, num_rounds: int) -> int:
        v = ctypes.c_int64()
        _native.check(_native.lib().qldpc_phenl_trace_len(self.handle, int(num_rounds), ctypes.byref(v)),
                      "qldpc_phenl_trace_len")
        return v.value

    def uniforms_per_sample(self, num_rounds: int) -> int:
        c = self.code
        return ((num_rounds - 1) * self.num_rep + 1) * (c.N + c.hx.shape[0] + c.hz.shape[0])

    def new_counters(self):
        torch = _torch()
        return torch.zeros(_native.COUNTER_WORDS, dtype=torch.int64, device=torch.device("cuda", self.device))

    def launch(self, px, py, pz, q, seed, shot_begin, shot_count, num_rounds, logical_mode="Total", counters=None,
               uniforms=None, fail=None, trace=None, stream=None):
        torch = _torch()
        if counters is None:
            raise ValueError("counters buffer required")
        mode = LOGICAL_MODES[logical_mode] if isinstance(logical_mode, str) else int(logical_mode)
        s = stream if stream is not None else _stream_handle(torch, counters.device)

        def ptr(t):
            return ctypes.c_void_p(t.data_ptr()) if t is not None else None

        _native.check(_native.lib().qldpc_phenl_launch(
            self.handle, float(px), float(py), float(pz), float(q), int(seed) & (2**64 - 1), int(shot_begin),
            int(shot_count), int(num_rounds), mode, ptr(uniforms), ptr(counters), ptr(fail), ptr(trace), s),
            "qldpc_phenl_launch")

    def run(self, px, py, pz, q, seed, shot_begin, shot_count, num_rounds, logical_mode="Total", uniforms=None,
            per_shot=False) -> MCResult:
        torch = _torch()
        dev = torch.device("cuda", self.device)
        S = int(shot_count)
        cnt = self.new_counters()
        u = None
        if uniforms is not None:
            u = torch.from_numpy(np.ascontiguousarray(uniforms, dtype=np.float64)).to(dev)
            if tuple(u.shape) != (S, self.uniforms_per_sample(num_rounds)):
                raise ValueError(f"uniforms must be [{S}, {self.uniforms_per_sample(num_rounds)}]")
        f = tr = None
        if per_shot:
            f = torch.zeros(S, dtype=torch.uint8, device=dev)
            tr = torch.zeros((S, self.trace_len(num_rounds)), dtype=torch.uint8, device=dev)
        self.launch(px, py, pz, q, seed, shot_begin, S, num_rounds, logical_mode, cnt, u, f, tr)
        torch.cuda.synchronize(dev)
        res = MCResult.from_words(cnt.cpu().numpy())
        if per_shot:
            res.fail = f.cpu().numpy()
            res.trace = tr.cpu().numpy()
        return res

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and _native._lib is not None:
            _native.lib().qldpc_phenl_destroy(h)
            self.handle = None


class DeviceCircuit:
    """Circuit-level space-time shot loop of ``CodeSimulator_Circuit_SpaceTime`` on one GPU
    (``qldpc_circ_*``, csrc/circuit.hip).

    ``dem`` is the FULL circuit's detector error model (:class:`~.circuit.DetectorErrorModel`),
    ``dec1`` decodes each round on h1 (num_rep·m rows), ``dec2`` the final layer on h2; ``hs``
    (h1_space_cor), ``L1`` and ``L2`` are dense 0/1 matrices as ``GenCorrecHyperGraph`` /
    ``GenFaultHyperGraph`` return them.  ``osd``: a :class:`DeviceOSD` (uniform priors) or a
    :class:`HostOSD` on h2 makes decoder2 BP+OSD (``dec2`` built with ``soft=True``).  ``sampler``:
    "skip" (default: geometric gaps per mechanism and global 64-sample word) or "keyed" (one Philox
    uniform per (sample, mechanism)); both exact and shard-invariant, different draws
    (``qldpc_circ_set_sampler``).
    """

    SAMPLERS = {"keyed": 0, "skip": 1}

    def __init__(self, dem, dec1: "DeviceBP | None" = None, hs=None, L1=None, dec2: "DeviceBP | None" = None, L2=None,
                 num_rounds: int = 0, num_rep: int = 1, osd=None, max_batch: int = 0, device: int | None = None,
                 sampler: str = "skip"):
        sampler_only = dec1 is None and dec2 is None
        if device is None:
            if dec1 is not None:
                device = dec1.graph.device
            else:
                from .parallel import local_device_index

                device = local_device_index()
        dev = device
        self.device = dev
        self.dem = dem
        self.decoders = (dec1, dec2)
        self.num_rounds, self.num_rep = int(num_rounds), int(num_rep)
        mats = [dem.check_matrix(), dem.observable_matrix()] + ([] if sampler_only else [hs, L1, L2])
        self._g = [DeviceGraph(np.asarray(a, dtype=np.uint8) % 2, device=dev) for a in mats]
        self._probs = np.ascontiguousarray(np.asarray(dem.probs, dtype=np.float64))
        hd = (lambda i: None) if sampler_only else (lambda i: self._g[i].handle)  # noqa: E731
        h = ctypes.c_void_p()
        _native.check(_native.lib().qldpc_circ_create(
            self._g[0].handle, self._g[1].handle, self._probs.ctypes.data_as(ctypes.c_void_p),
            None if sampler_only else dec1.handle, hd(2), hd(3), None if sampler_only else dec2.handle, hd(4),
            self.num_rounds, self.num_rep, int(max_batch), ctypes.byref(h)), "qldpc_circ_create")
        self.handle = h
        self.sampler = sampler
        _native.check(_native.lib().qldpc_circ_set_sampler(h, self.SAMPLERS[sampler]), "qldpc_circ_set_sampler")
        self._osd = osd
        if osd is not None:
            gpu = osd.handle if isinstance(osd, DeviceOSD) else None
            host = osd.handle if isinstance(osd, HostOSD) else None
            _native.check(_native.lib().qldpc_circ_set_final_osd(h, gpu, host), "qldpc_circ_set_final_osd")

    @property
    def num_detectors(self) -> int:
        return self.dem.num_detectors

    @property
    def num_observables(self) -> int:
        return self.dem.num_observables

    def new_counters(self):
        torch = _torch()
        return torch.zeros(_native.COUNTER_WORDS, dtype=torch.int64, device=torch.device("cuda", self.device))

    def launch(self, seed, shot_begin, shot_count, counters, fail=None, detobs=None, stream=None):
        torch = _torch()
        s = stream if stream is not None else _stream_handle(torch, counters.device)

        def ptr(t):
            return ctypes.c_void_p(t.data_ptr()) if t is not None else None

        _native.check(_native.lib().qldpc_circ_launch(self.handle, int(seed) & (2**64 - 1), int(shot_begin),
                                                      int(shot_count), ptr(counters), ptr(fail), ptr(detobs), s),
                      "qldpc_circ_launch")

    def sample(self, seed, shot_begin, shot_count):
        """Detector + observable bits [S, D + K] (uint8, host) of samples ``shot_begin..`` — the
        ``detector_sampler.sample(shots, append_observables=True)`` of the reference."""
        torch = _torch()
        dev = torch.device("cuda", self.device)
        S = int(shot_count)
        out = torch.zeros((S, self.num_detectors + self.num_observables), dtype=torch.uint8, device=dev)
        _native.check(_native.lib().qldpc_circ_sample(self.handle, int(seed) & (2**64 - 1), int(shot_begin), S,
                                                      ctypes.c_void_p(out.data_ptr()), _stream_handle(torch, dev)),
                      "qldpc_circ_sample")
        torch.cuda.synchronize(dev)
        return out.cpu().numpy()

    def run(self, seed, shot_begin, shot_count, per_shot: bool = False) -> "MCResult":
        """Counters of ``shot_count`` samples (``per_shot``: also ``fail`` [S] and the sampled
        detector / observable bits ``detobs`` [S, D + K] as host arrays)."""
        torch = _torch()
        dev = torch.device("cuda", self.device)
        cnt = self.new_counters()
        S = int(shot_count)
        fail = torch.zeros(S, dtype=torch.uint8, device=dev) if per_shot else None
        detobs = torch.zeros((S, self.num_detectors + self.num_observables), dtype=torch.uint8, device=dev) \
            if per_shot else None
        self.launch(seed, shot_begin, S, cnt, fail, detobs)
        torch.cuda.synchronize(dev)
        res = MCResult.from_words(cnt.cpu().numpy())
        if per_shot:
            res.fail = fail.cpu().numpy()
            res.detobs = detobs.cpu().numpy()
        return res

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and _native._lib is not None:
            _native.lib().qldpc_circ_destroy(h)
            self.handle = None
