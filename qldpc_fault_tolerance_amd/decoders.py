"""Drop-in decoder classes with the reference's names and signatures.

Mirrors ``src/Decoders.py`` and the space-time part of
``src/Decoders_SpaceTime.py``.  Where the reference wraps the third-party
``ldpc.bp_decoder`` (``src/Decoders.py:77-90``), these classes wrap the MI355X
BP engine (:class:`engine.DeviceBP`): same constructor arguments, same
``decode(synd) -> ndarray[int]`` contract, plus ``decode_batch`` for many
syndromes per launch.  ``device=None`` (the default everywhere) resolves to this
process's GPU: ``LOCAL_RANK`` under ``torch.distributed.run`` (one rank per GPU),
else 0 (:func:`.parallel.local_device_index`).  ``DecoderClass.GetDecoder(params)`` keeps the reference's
dict keys and assertions (``:94-172``; ``src/Decoders_SpaceTime.py:227-257``).

BP+OSD (``BPOSD_Decoder``): GPU BP with soft output, then
the native OSD stage (csrc/osd.hip) on the syndromes BP did not converge on.
"""
from __future__ import annotations

import math
from abc import ABC, abstractmethod

import numpy as np

from .codes import CSR, space_time_csr


def _int_max_iter(max_iter, n):
    # ldpc stores max_iter in a C int: the float n/max_iter_ratio the factories
    # pass (src/Decoders.py:123,162 — quirk Q1) is truncated; 0 means n.
    mi = int(max_iter)
    return mi if mi > 0 else n


class BPDecoder:
    """``BPDecoder(h, channel_probs, max_iter, bp_method, ms_scaling_factor)`` (``src/Decoders.py:77-90``)."""

    def __init__(self, h, channel_probs, max_iter, bp_method, ms_scaling_factor, precision: int = 64,
                 device: int | None = None, vars_per_thread: int = 0):
        from .engine import DeviceBP

        self.h = h
        self.max_iter = max_iter
        self.bp_method = bp_method
        self.ms_scaling_factor = ms_scaling_factor
        self.channel_probs = np.asarray(channel_probs, dtype=np.float64)
        H = h if isinstance(h, CSR) else CSR.from_dense(h)
        self.num_checks, self.num_qubits = H.m, H.n
        self.decoder = DeviceBP(H, self.channel_probs, max_iter=_int_max_iter(max_iter, H.n), bp_method=bp_method,
                                ms_scaling_factor=ms_scaling_factor, precision=precision, device=device,
                                vars_per_thread=vars_per_thread)
        self.iter = 0
        self.converge = 0

    def decode(self, synd):
        corr, it, conv = self.decoder.decode_batch(np.asarray(synd).reshape(1, -1))
        self.iter, self.converge = int(it[0]), int(conv[0])
        return corr[0]

    def decode_batch(self, synd):
        """[B, m] syndromes -> ([B, n] corrections, iterations [B], converged [B])."""
        return self.decoder.decode_batch(synd)


class FirstMinBPDecoder:
    """Repeated one-iteration BP while the syndrome weight does not grow (``src/Decoders.py:49-74``).

    ``minimum_sum`` (every reference call site) runs the whole loop on the GPU in one kernel
    (:class:`~.engine.DeviceFirstMin`, ``qldpc_firstmin_*``); ``product_sum``, and graphs past that
    kernel's envelope (2 (m + n) > 64 KiB: ``QLDPC_ENOTSUP``), step the engine's one-iteration BP
    from the host (one launch per first-min step for all active syndromes).  ``max_iter`` is
    compared raw, as ``iter_counter < self.max_iter`` (``:66``): a float N/10 = 22.5 allows 23
    accepted steps, so the device loop takes ``ceil(max_iter)``."""

    def __init__(self, h, channel_probs, max_iter, bp_method, ms_scaling_factor, precision: int = 64,
                 device: int | None = None):
        from . import _native
        from .engine import DeviceFirstMin, bp_method_code

        self.h = np.asarray(h)
        self.max_iter = max_iter
        self._H = CSR.from_dense(self.h)
        self._fm = None
        self._bp = None
        if bp_method_code(bp_method) == 1:
            n = self._H.n
            probs = np.asarray(channel_probs, dtype=np.float64)
            try:
                self._fm = DeviceFirstMin(self._H, np.full(n, float(probs)) if probs.ndim == 0 else probs,
                                          max(0, math.ceil(max_iter)), ms_scaling_factor, precision=precision,
                                          device=device)
            except _native.QldpcError as e:
                if e.rc != _native.ENOTSUP:
                    raise
        if self._fm is None:
            self._bp = BPDecoder(h, channel_probs, 1, bp_method, ms_scaling_factor, precision=precision, device=device)
        self.steps_batch = None
        self._st_bp = None
        self._probs = np.asarray(channel_probs, dtype=np.float64)

    def st_bp(self):
        """A one-iteration engine BP on this decoder's own device graph: the slot the fused
        phenomenological pipeline validates its space-time graph against (its decodes are replaced
        by this decoder's first-min loop, qldpc_phenl_set_round_firstmin)."""
        if self._st_bp is None:
            from .engine import DeviceBP

            n = self._H.n
            p = np.full(n, float(self._probs)) if self._probs.ndim == 0 else self._probs
            self._st_bp = DeviceBP(self._H, p, max_iter=1, graph=self._fm.graph if self._fm is not None else None)
        return self._st_bp

    def decode(self, synd):
        return self.decode_batch(np.asarray(synd).reshape(1, -1))[0]

    def decode_batch(self, synd):
        """[B, m] syndromes -> [B, n] corrections (int64); ``steps_batch`` = accepted steps."""
        if self._fm is not None:
            corr, self.steps_batch = self._fm.decode_batch(synd)
            return corr
        return self._decode_batch_stepped(synd)

    def _decode_batch_stepped(self, synd):
        S = (np.atleast_2d(np.asarray(synd)).astype(np.int64) % 2).astype(np.uint8)
        B = S.shape[0]
        correction = np.zeros((B, self._H.n), dtype=np.int64)
        current = S.copy()
        active = np.ones(B, dtype=bool)
        counter = np.zeros(B, dtype=np.int64)
        new_corr, _, _ = self._bp.decode_batch(current)
        new_synd = (self._H.matvec(new_corr.astype(np.uint8)) ^ current).astype(np.uint8)
        while True:
            ok = active & (new_synd.sum(1) <= current.sum(1)) & (counter < self.max_iter)
            if not ok.any():
                break
            current[ok] = new_synd[ok]
            correction[ok] = (correction[ok] + new_corr[ok]) % 2
            counter[ok] += 1
            active = ok
            idx = np.flatnonzero(ok)
            nc, _, _ = self._bp.decode_batch(current[idx])
            new_corr[idx] = nc
            new_synd[idx] = (self._H.matvec(nc.astype(np.uint8)) ^ current[idx]).astype(np.uint8)
        return correction


class BPOSD_Decoder:
    """``BPOSD_Decoder(h, channel_probs, max_iter, bp_method, ms_scaling_factor, osd_method, osd_order)``
    (``src/Decoders.py:26-41``): ``bposd_decoder`` = BP, then OSD when BP does not converge.

    BP runs on the GPU (engine 1 with soft output: ``qldpc_bp_decode_batch_soft``)
    and hands its final posteriors to the native OSD stage (``qldpc_osd_decode_batch``).
    ``decode`` returns ``osdw_decoding`` like the reference; ``osd0_decoding``,
    ``bp_decoding``, ``converge``, ``iter`` and ``log_prob_ratios`` are kept.
    """

    def __init__(self, h, channel_probs, max_iter, bp_method, ms_scaling_factor, osd_method, osd_order,
                 precision: int = 64, device: int | None = None, osd_threads: int = 0, use_gpu_osd: bool = True):
        from .engine import DeviceBP, DeviceOSD, HostOSD

        self.h = h
        H = h if isinstance(h, CSR) else CSR.from_dense(h)
        self.num_checks, self.num_qubits = H.m, H.n
        self.channel_probs = np.asarray(channel_probs, dtype=np.float64)
        self.osd_method, self.osd_order = osd_method, osd_order
        self.decoder = DeviceBP(H, self.channel_probs, max_iter=_int_max_iter(max_iter, H.n), bp_method=bp_method,
                                ms_scaling_factor=ms_scaling_factor, precision=precision, device=device, soft=True)
        self.osd = HostOSD(H, self.channel_probs, osd_method=osd_method, osd_order=osd_order)
        # OSD on the GPU (uniform priors: popcount weights; non-uniform: soft weights); the host stage
        # stays for use_gpu_osd=False and graphs past the GPU kernel's envelope
        self.gpu_osd = (DeviceOSD(self.decoder.graph, self.channel_probs, osd_method, osd_order)
                        if use_gpu_osd and DeviceOSD.supported(H.n, self.channel_probs, osd_method, osd_order)
                        else None)
        self.osd_threads = osd_threads
        self.iter, self.converge = 0, 0

    def decode_batch(self, synd):
        """[B, m] syndromes -> osdw corrections [B, n] (int); also sets the batch's
        ``osd0_batch``, ``bp_batch``, ``conv_batch``, ``iters_batch``, ``post_batch`` (the
        posteriors; a device tensor when the OSD ran on the GPU)."""
        s = np.atleast_2d(np.asarray(synd))
        if self.gpu_osd is not None:
            ow, o0, corr, iters, conv, post = self.gpu_osd.bposd_batch(self.decoder, s, host_post=False)
        else:
            corr, iters, conv, post = self.decoder.decode_batch_soft(s)
            o0, ow = self.osd.decode_batch(s, post, conv, corr, threads=self.osd_threads)
        self.bp_batch, self.iters_batch, self.conv_batch, self.post_batch = corr, iters, conv, post
        self.osd0_batch = o0.astype(np.int64)
        return ow.astype(np.int64)

    def decode(self, synd):
        ow = self.decode_batch(np.asarray(synd).reshape(1, -1))
        self.bp_decoding = self.bp_batch[0]
        self.osd0_decoding = self.osd0_batch[0]
        self.osdw_decoding = ow[0]
        pb = self.post_batch
        self.log_prob_ratios = pb[0] if isinstance(pb, np.ndarray) else pb[0].cpu().numpy()
        self.iter, self.converge = int(self.iters_batch[0]), int(self.conv_batch[0])
        return self.osdw_decoding


class DecoderClass(ABC):
    """``src/Decoders.py:94-97``."""

    @abstractmethod
    def GetDecoder(self, code_and_noise_channel_params):
        pass


class BP_Decoder_Class(DecoderClass):
    """``src/Decoders.py:141-172``: factory keyed by ``{'h', 'p_data'[, 'p_syndrome']}``."""

    def __init__(self, max_iter_ratio: int, bp_method: str, ms_scaling_factor: float, precision: int = 64,
                 device: int | None = None):
        self.decoder_default_params = {"max_iter_ratio": max_iter_ratio, "bp_method": bp_method,
                                       "ms_scaling_factor": ms_scaling_factor}
        self.precision = precision
        self.device = device

    @staticmethod
    def _probs(params):
        h = params["h"]
        if "p_syndrome" in params:
            num_checks, num_qubits = h.shape[0], h.shape[1] - h.shape[0]
            probs = np.hstack([params["p_data"] * np.ones(num_qubits), params["p_syndrome"] * np.ones(num_checks)])
        else:
            num_checks, num_qubits = h.shape
            probs = params["p_data"] * np.ones(num_qubits)
        return num_qubits, probs

    def GetDecoder(self, code_and_noise_channel_params):
        p = code_and_noise_channel_params
        assert "h" in p.keys(), "missing the check matrix h"
        assert "p_data" in p.keys(), "missing the data error prob: p_data"
        num_qubits, probs = self._probs(p)
        max_iter = num_qubits / self.decoder_default_params["max_iter_ratio"]
        return BPDecoder(h=p["h"], channel_probs=probs, max_iter=max_iter,
                         bp_method=self.decoder_default_params["bp_method"],
                         ms_scaling_factor=self.decoder_default_params["ms_scaling_factor"],
                         precision=self.precision, device=self.device)


class BPOSD_Decoder_Class(DecoderClass):
    """``src/Decoders.py:100-138``: BP+OSD factory keyed like :class:`BP_Decoder_Class`."""

    def __init__(self, max_iter_ratio: int, bp_method: str, ms_scaling_factor: float, osd_method: str,
                 osd_order: int, precision: int = 64, device: int | None = None):
        self.decoder_default_params = {"max_iter_ratio": max_iter_ratio, "bp_method": bp_method,
                                       "ms_scaling_factor": ms_scaling_factor, "osd_method": osd_method,
                                       "osd_order": osd_order}
        self.precision = precision
        self.device = device

    def GetDecoder(self, code_and_noise_channel_params):
        p = code_and_noise_channel_params
        assert "h" in p.keys(), "missing the check matrix h"
        assert "p_data" in p.keys(), "missing the data error prob: p_data"
        num_qubits, probs = BP_Decoder_Class._probs(p)
        d = self.decoder_default_params
        max_iter = num_qubits / d["max_iter_ratio"]
        return BPOSD_Decoder(h=p["h"], channel_probs=probs, max_iter=max_iter, bp_method=d["bp_method"],
                             ms_scaling_factor=d["ms_scaling_factor"], osd_method=d["osd_method"],
                             osd_order=d["osd_order"], precision=self.precision, device=self.device)


# ------------------------------------------------------------------ space-time
def GetSpaceTimeCheckMat(h, t0):
    """Dense ``t0·m × t0·(n+m)`` space-time check matrix (``src/Decoders_SpaceTime.py:179-194``)."""
    H = np.asarray(h)
    return space_time_csr(H, int(t0)).to_dense().astype(np.float64)


def fold_space_time_correction(error_history, num_qubits: int, num_checks: int, num_rep: int):
    """Sum of the data slices of a space-time decoding, mod 2 (``src/Decoders_SpaceTime.py:218-223``)."""
    E = np.asarray(error_history)
    w = num_qubits + num_checks
    lead = E.shape[:-1]
    E = E.reshape(lead + (num_rep, w))
    return (E[..., :num_qubits].astype(np.int64).sum(axis=-2) % 2)


class ST_BP_Decoder_syndrome:
    """BP on the stacked space-time graph (``src/Decoders_SpaceTime.py:200-223``)."""

    def __init__(self, h, p_data: float, p_synd: float, max_iter: int, bp_method: str, ms_scaling_factor,
                 num_rep: int, precision: int = 64, device: int | None = None):
        from .engine import DeviceBP

        H = np.asarray(h)
        self.num_checks, self.num_qubits = H.shape
        self.h = H
        self.num_rep = int(num_rep)
        self.ST_csr = space_time_csr(H, self.num_rep)
        probs = np.hstack([p_data * np.ones(self.num_qubits), p_synd * np.ones(self.num_checks)] * self.num_rep)
        self.channel_probs = probs
        self.max_iter = max_iter
        self.space_decoder = DeviceBP(self.ST_csr, probs, max_iter=_int_max_iter(max_iter, self.ST_csr.n),
                                      bp_method=bp_method, ms_scaling_factor=ms_scaling_factor, precision=precision,
                                      device=device)

    @property
    def ST_h(self):
        return self.ST_csr.to_dense().astype(np.float64)

    def decode(self, detector_history):
        return self.decode_batch(np.asarray(detector_history)[None])[0]

    def decode_batch(self, detector_histories):
        """[B, num_rep, m] detector histories -> [B, n] corrections."""
        D = np.asarray(detector_histories)
        B = D.shape[0]
        synd = D.reshape(B, D.shape[1] * D.shape[2])
        err, _, _ = self.space_decoder.decode_batch(synd)
        return fold_space_time_correction(err, self.num_qubits, self.num_checks, self.num_rep)


class ST_BP_Decoder_Class(DecoderClass):
    """``src/Decoders_SpaceTime.py:227-257`` (keeps quirk Q4: p_synd = p_data when p_syndrome is given)."""

    def __init__(self, max_iter_ratio: int, bp_method: str, ms_scaling_factor: float, precision: int = 64,
                 device: int | None = None):
        self.decoder_default_params = {"max_iter_ratio": max_iter_ratio, "bp_method": bp_method,
                                       "ms_scaling_factor": ms_scaling_factor}
        self.precision = precision
        self.device = device

    def GetDecoder(self, code_and_noise_channel_params):
        p = code_and_noise_channel_params
        assert "h" in p.keys(), "missing the check matrix h"
        assert "p_data" in p.keys(), "missing the data error prob: p_data"
        assert "num_rep" in p.keys(), "missing the data error prob: p_data"
        h = p["h"]
        p_data = p["p_data"]
        num_checks, num_qubits = np.asarray(h).shape
        p_synd = p["p_data"] if "p_syndrome" in p.keys() else 0
        max_iter = num_qubits / self.decoder_default_params["max_iter_ratio"]
        return ST_BP_Decoder_syndrome(h=h, p_data=p_data, p_synd=p_synd, max_iter=max_iter,
                                      bp_method=self.decoder_default_params["bp_method"],
                                      ms_scaling_factor=self.decoder_default_params["ms_scaling_factor"],
                                      num_rep=p["num_rep"], precision=self.precision, device=self.device)


# ------------------------------------------------------------------ circuit-level space-time
class ST_BP_Decoder_Circuit(BPDecoder):
    """``ST_BP_Decoder_Circuit(h, channel_probs, max_iter, bp_method, ms_scaling_factor)``
    (``src/Decoders_SpaceTime.py:261-274``): BP on a fault hypergraph (``GenFaultHyperGraph``'s h1),
    ``decode`` returns the correction mod 2.  ``h`` has a column per DEM error mechanism and
    non-uniform ``channel_probs`` (the mechanisms' probabilities)."""

    def __init__(self, h, channel_probs, max_iter, bp_method, ms_scaling_factor, precision: int = 64,
                 device: int | None = None):
        super().__init__(h, channel_probs, max_iter, bp_method, ms_scaling_factor, precision=precision,
                         device=device)
        self.space_decoder = self.decoder

    def decode(self, synd):
        return super().decode(synd) % 2


class ST_BPOSD_Decoder_Circuit(BPOSD_Decoder):
    """``ST_BPOSD_Decoder_Circuit(h, channel_probs, max_iter, bp_method, ms_scaling_factor, osd_method,
    osd_order)`` (``src/Decoders_SpaceTime.py:277-292``): ``bposd_decoder`` on h2; ``decode`` returns
    ``osdw_decoding``.  DEM priors are non-uniform: the GPU OSD weighs its candidates by
    sum log(1/p_j) (the host stage's order relation, summed in the same column order)."""


class ST_BP_Decoder_Circuit_Class(DecoderClass):
    """``src/Decoders_SpaceTime.py:296-321``: keys ``h``, ``code_h``, ``channel_probs``;
    ``max_iter = int(n(code_h) / max_iter_ratio)``."""

    def __init__(self, max_iter_ratio: int, bp_method: str, ms_scaling_factor: float, precision: int = 64):
        self.decoder_default_params = {"max_iter_ratio": max_iter_ratio, "bp_method": bp_method,
                                       "ms_scaling_factor": ms_scaling_factor}
        self.precision = precision

    def GetDecoder(self, code_and_noise_channel_params):
        p = code_and_noise_channel_params
        assert "h" in p.keys(), "missing the check matrix h"
        assert "code_h" in p.keys(), "missing the code"
        assert "channel_probs" in p.keys(), "missing the channel_probs"
        _, num_qubits = np.shape(p["code_h"])
        d = self.decoder_default_params
        return ST_BP_Decoder_Circuit(h=p["h"], channel_probs=p["channel_probs"],
                                     max_iter=int(num_qubits / d["max_iter_ratio"]), bp_method=d["bp_method"],
                                     ms_scaling_factor=d["ms_scaling_factor"], precision=self.precision)


class ST_BPOSD_Decoder_Circuit_Class(DecoderClass):
    """``src/Decoders_SpaceTime.py:323-357``: a ``BPOSD_Decoder`` on ``h`` with ``max_iter =
    n(code_h) / max_iter_ratio`` passed as a float (quirk Q1: truncated by ldpc)."""

    def __init__(self, max_iter_ratio: int, bp_method: str, ms_scaling_factor: float, osd_method: str,
                 osd_order: int, precision: int = 64):
        self.decoder_default_params = {"max_iter_ratio": max_iter_ratio, "bp_method": bp_method,
                                       "ms_scaling_factor": ms_scaling_factor, "osd_method": osd_method,
                                       "osd_order": osd_order}
        self.precision = precision

    def GetDecoder(self, code_and_noise_channel_params):
        p = code_and_noise_channel_params
        assert "h" in p.keys(), "missing the check matrix h"
        assert "code_h" in p.keys(), "missing the code"
        assert "channel_probs" in p.keys(), "missing the channel_probs"
        _, num_qubits = np.shape(p["code_h"])
        d = self.decoder_default_params
        return BPOSD_Decoder(h=p["h"], channel_probs=p["channel_probs"], max_iter=num_qubits / d["max_iter_ratio"],
                             bp_method=d["bp_method"], ms_scaling_factor=d["ms_scaling_factor"],
                             osd_method=d["osd_method"], osd_order=d["osd_order"], precision=self.precision)
