"""Drop-in Monte Carlo simulators with the reference's names and signatures.

Mirrors the code-capacity part of ``src/Simulators.py``:

* :class:`CodeSimulator_DataError` (``:75-188``) — ``WordErrorRate(num_run)``
  returns ``(wer, wer_eb)`` with the reference's formulas (incl. quirk Q2).
  When both decoders are this engine's :class:`~.decoders.BPDecoder`, the shot
  loop runs as ONE fused HIP launch per GPU (sample → syndrome → BP →
  residual → logical check, ``qldpc_mc_launch``), shots sharded over the
  ``torch.distributed`` ranks with a single counter all-reduce
  (:mod:`.parallel`).  Decoders from elsewhere (any object with
  ``.decode(synd)``, the reference's plugin contract ``src/Decoders.py:94-97``)
  run through the per-shot ``_single_run`` loop, as in the reference.
* :class:`CodeFamily` (``:746-908``) — ``EvalWER('data', ...)``.
* the threshold-fit helpers (``:675-741``), host-side post-processing.

Shot randomness: the reference draws ``random.random()`` per qubit (MT19937,
re-seeded per forked worker, so not reproducible).  The fused path draws the
same 53-bit uniforms from Philox4x32-10 keyed by ``(seed, global shot, qubit)``
— reproducible and identical for any GPU count; ``seed`` defaults to 64 bits
of Python's ``random`` so ``random.seed(s)`` still pins a run.
"""
from __future__ import annotations

import random

import numpy as np

from . import parallel
from .codes import load_code

# ------------------------------------------------------------------ formulas


def pauli_split(u, pauli_error_probs):
    """Reference 3-way split of uniforms ``u`` (``src/Simulators.py:99-113``) -> (e_x, e_z) int arrays.

    ``pauli_error_probs = [px, py, pz]``: Z if ``u < pz``; X if ``pz <= u < pz+px``;
    Y (both) if ``pz+px <= u < pz+px+py`` — thresholds summed in that order.
    """
    px, py, pz = (float(x) for x in pauli_error_probs)
    u = np.asarray(u, dtype=np.float64)
    t1, t2, t3 = pz, pz + px, (pz + px) + py
    z_only = u < t1
    x_only = (t1 <= u) & (u < t2)
    y = (t2 <= u) & (u < t3)
    e_x = (x_only | y).astype(np.int64)
    e_z = (z_only | y).astype(np.int64)
    return e_x, e_z


def word_error_rate(error_count: int, num_run: int, K: int):
    """``WordErrorRate`` arithmetic of ``src/Simulators.py:174-188`` (keeps quirk Q2: ``eb`` for LER)."""
    ler = error_count / num_run
    ler_eb = np.sqrt((1 - ler) * ler / num_run)
    wer = 1.0 - (1 - ler) ** (1 / K)
    wer_eb = ler_eb * ((1 - ler_eb) ** (1 / K - 1)) / K
    return wer, wer_eb


def word_error_rate_per_cycle(error_count: int, num_samples: int, K: int, total_num_cycles: int):
    """Per-qubit per-cycle WER of the multi-round simulators (``src/Simulators_SpaceTime.py:538-548``)."""
    assert int(total_num_cycles) % 2 == 1
    ler = error_count / num_samples
    ler_q = 1.0 - (1 - ler) ** (1 / K)
    if ler_q <= 0.5:
        return (1.0 - (1 - 2 * ler_q) ** (1 / total_num_cycles)) / 2
    return (1.0 + (-1 + 2 * ler_q) ** (1 / total_num_cycles)) / 2


def load_object(filename):
    """``load_object`` (``src/Simulators.py:69-71``) for code files, without unpickling."""
    return load_code(filename)


# --------------------------------------------------------------- simulators


def _engine_bp(decoder):
    """The engine's DeviceBP behind a drop-in decoder, or None for a foreign decoder."""
    from .engine import DeviceBP

    if getattr(decoder, "osd", None) is not None:  # BPOSD_Decoder: OSD runs after BP, per-shot path
        return None
    bp = getattr(decoder, "decoder", None)
    return bp if isinstance(bp, DeviceBP) else None


def _final_round_bp(decoder):
    """DeviceBP of a final-round decoder: an engine BPDecoder, or a BPOSD_Decoder whose OSD
    runs on the GPU (its soft BP then feeds qldpc_phenl_set_final_osd)."""
    if _is_bposd(decoder):
        return decoder.decoder if getattr(decoder, "gpu_osd", None) is not None else None
    return _engine_bp(decoder)


def _is_bposd(decoder) -> bool:
    return getattr(decoder, "osd", None) is not None


def gf2_rows(csr, X):
    """Rows of ``X`` [S, n] (0/1) times ``H^T`` mod 2 -> [S, m] uint8, for a :class:`~.codes.CSR` ``H``
    (sparse x sparse: the error / residual rows are sparse)."""
    import scipy.sparse as sp

    Ht = getattr(csr, "_gf2_ht", None)
    if Ht is None:
        Ht = sp.csr_matrix((np.ones(len(csr.col_idx), np.int32), np.asarray(csr.col_idx), np.asarray(csr.row_ptr)),
                           shape=(csr.m, csr.n)).T.tocsc()
        csr._gf2_ht = Ht
    X = np.asarray(X)
    if X.shape[0] == 0:
        return np.zeros((0, csr.m), dtype=np.uint8)
    P = sp.csr_matrix(X.astype(np.int32, copy=False)) @ Ht
    return (P.toarray() & 1).astype(np.uint8)


class CodeSimulator_DataError:
    """Data-error simulator (``src/Simulators.py:75-188``).

    Extra keyword arguments (not in the reference): ``seed`` for the fused
    path's Philox stream.
    """

    def __init__(self, code=None, decoder_x=None, decoder_z=None, pauli_error_probs=(0.01, 0.01, 0.01),
                 eval_logical_type="Total", seed=None):
        self.code = code
        self.decoder_z, self.decoder_x = decoder_z, decoder_x
        self.N = code.N
        self.K = code.K
        self.channel_probs = list(pauli_error_probs)
        self.error_x = np.zeros(self.N).astype(int)
        self.error_z = np.zeros(self.N).astype(int)
        self.min_logical_weight = self.N
        self.eval_logical_type = eval_logical_type
        self.seed = int(seed) if seed is not None else None
        self._shot_offset = 0
        self._mc = None
        self.last_result = None

    # -- reference per-shot API (plugin path) --------------------------------
    def _generate_error(self):
        u = np.array([random.random() for _ in range(self.N)])
        self.error_x, self.error_z = pauli_split(u, self.channel_probs)
        return self.error_x, self.error_z

    def _single_run(self):
        self.error_x, self.error_z = self._generate_error()
        code = self.code
        synd_z = code.hx @ self.error_z % 2
        decoded_z = self.decoder_z.decode(synd_z)
        synd_x = code.hz @ self.error_x % 2
        decoded_x = self.decoder_x.decode(synd_x)
        residual_x = (self.error_x + decoded_x) % 2
        residual_z = (self.error_z + decoded_z) % 2
        X_failure = int(((code.hz @ residual_x) % 2).any() or ((code.lz @ residual_x) % 2).any())
        Z_failure = int(((code.hx @ residual_z) % 2).any() or ((code.lx @ residual_z) % 2).any())
        for fail, r, L in ((X_failure, residual_x, code.lz), (Z_failure, residual_z, code.lx)):
            if fail and ((L @ r) % 2).any():
                self.min_logical_weight = min(self.min_logical_weight, int(np.sum(r)))
        assert self.eval_logical_type in ["X", "Z", "Total"]
        if self.eval_logical_type == "X":
            return X_failure
        if self.eval_logical_type == "Z":
            return Z_failure
        return X_failure or Z_failure

    # -- fused engine path ----------------------------------------------------
    def _engine_ready(self):
        need_x = self.eval_logical_type != "Z"
        need_z = self.eval_logical_type != "X"
        bx = _engine_bp(self.decoder_x) if need_x else None
        bz = _engine_bp(self.decoder_z) if need_z else None
        return (not need_x or bx is not None) and (not need_z or bz is not None), bx, bz

    def _device_mc(self, bx, bz):
        from .engine import DeviceMC

        if self._mc is None:
            self._mc = DeviceMC(self.code, bx, bz)
        return self._mc

    def fused_counts(self, num_run: int):
        """Run ``num_run`` shots through the fused HIP path; returns the all-reduced :class:`~.engine.MCResult`."""
        ok, bx, bz = self._engine_ready()
        if not ok:
            raise TypeError("fused path needs engine BPDecoder instances for the sectors eval_logical_type uses")
        from .engine import MCResult, _torch

        torch = _torch()
        if self.seed is None:
            self.seed = random.getrandbits(64)
        mc = self._device_mc(bx, bz)
        rank, ws = parallel.world()
        b, c = parallel.shard_range(num_run, rank, ws, begin=self._shot_offset)
        self._shot_offset += int(num_run)
        px, py, pz = self.channel_probs
        cnt = mc.new_counters()
        mc.launch(px, py, pz, self.seed, b, c, self.eval_logical_type, cnt)
        parallel.allreduce_counters(cnt)
        torch.cuda.synchronize(cnt.device)
        res = MCResult.from_words(cnt.cpu().numpy())
        self.last_result = res
        return res

    # -- BP+OSD shot loop ---------------------------------------------------------
    def _bposd_ready(self):
        need_x = self.eval_logical_type != "Z"
        need_z = self.eval_logical_type != "X"
        return (not need_x or _is_bposd(self.decoder_x)) and (not need_z or _is_bposd(self.decoder_z))

    def bposd_counts(self, num_run: int, batch: int = 1 << 18, keep_shots: bool = False):
        """``num_run`` shots with BPOSD_Decoder sectors (the notebooks' decoder,
        src/Decoders.py:26-41) -> (failures, shots, osd_decodes), all-reduced.

        Device-resident when both sectors' OSD runs on the GPU (uniform priors, every reference
        call site): per batch ONE fused launch samples, decodes with engine-3 BP built on the
        BPOSD decoders' own graphs and parameters, captures every decode that reaches max_iter
        without converging (its posteriors, syndrome and error), runs the GPU OSD stage on those
        and re-checks their residuals, all on the device (``qldpc_mc_set_osd``); converged decodes
        keep the BP verdict, exactly as ``bposd_decoder`` returns the BP decoding when BP
        converges.  Otherwise the host-assisted path below.  ``keep_shots`` stores ``last_shots``
        = (errors [S, n] bit0 x / bit1 z, sector failures [S, 2]).
        """
        if not self._bposd_ready():
            raise TypeError("bposd_counts needs BPOSD_Decoder instances for the sectors eval_logical_type uses")
        need_x = self.eval_logical_type != "Z"
        need_z = self.eval_logical_type != "X"
        decs = [d for d, need in ((self.decoder_x, need_x), (self.decoder_z, need_z)) if need]
        if all(getattr(d, "gpu_osd", None) is not None for d in decs) and self._bposd_device_mc(need_x, need_z):
            return self._bposd_counts_device(num_run, batch, keep_shots, need_x, need_z)
        return self._bposd_counts_host(num_run, min(int(batch), 16384), keep_shots)

    def _bposd_device_mc(self, need_x, need_z):
        """The device-resident BP+OSD loop needs the fused engine-3 MC kernel
        (``qldpc_mc_set_osd``); graphs outside its envelope, a forced engine
        (``QLDPC_ENGINE``) or the staged pipeline (``QLDPC_MC_STAGED=1``) keep the
        host-assisted loop.  Returns the MC handle, or None (decided once)."""
        if getattr(self, "_bposd_dev", None) is None:
            from ._native import QldpcError
            from .engine import DeviceBP, DeviceMC

            def fast(dec, vpl=0):
                b = dec.decoder  # the soft (engine-1) BP: same graph, priors, max_iter, alpha, precision
                return DeviceBP(None, b.channel_probs, max_iter=b.max_iter, bp_method="minimum_sum",
                                ms_scaling_factor=b.ms_scaling_factor, precision=b.precision, graph=b.graph,
                                vars_per_thread=vpl)

            self._bposd_dev = False
            # the fused kernel is min-sum: product-sum BP+OSD decoders keep the host-assisted loop
            if any(d.decoder.bp_method != 1 for d, need in ((self.decoder_x, need_x), (self.decoder_z, need_z))
                   if need):
                return None
            bx = fast(self.decoder_x) if need_x else None
            # one fused kernel serves both sectors: the Z sector takes the X sector's geometry
            bz = fast(self.decoder_z, bx.geometry()["vars_per_thread"] if bx is not None else 0) if need_z else None
            if all(b is None or b.geometry()["engine"] == 3 for b in (bx, bz)):
                mc = DeviceMC(self.code, bx, bz)
                try:
                    mc.set_osd(self.decoder_x.gpu_osd if need_x else None,
                               self.decoder_z.gpu_osd if need_z else None)
                    self._bposd_dev = mc
                except QldpcError:  # staged MC or another engine: the host-assisted loop
                    pass
        return self._bposd_dev or None

    def _bposd_counts_device(self, num_run, batch, keep_shots, need_x, need_z):
        from .engine import MCResult, _torch

        torch = _torch()
        if self.seed is None:
            self.seed = random.getrandbits(64)
        mc = self._bposd_dev
        rank, ws = parallel.world()
        b, c = parallel.shard_range(num_run, rank, ws, begin=self._shot_offset)
        self._shot_offset += int(num_run)
        px, py, pz = self.channel_probs
        dev = torch.device("cuda", mc.device)
        cnt = mc.new_counters()
        kept_e, kept_f = [], []
        for s0 in range(b, b + c, int(batch)):
            S = min(int(batch), b + c - s0)
            f_d = e_d = None
            if keep_shots:
                f_d = torch.zeros(S, dtype=torch.uint8, device=dev)
                e_d = torch.zeros((S, self.N), dtype=torch.uint8, device=dev)
            mc.launch(px, py, pz, self.seed, s0, S, self.eval_logical_type, cnt, None, f_d, e_d)
            if keep_shots:
                f = f_d.cpu().numpy()
                kept_e.append(e_d.cpu().numpy())
                kept_f.append(np.stack([(f & 1) != 0, (f & 2) != 0], axis=1))
        if keep_shots:
            self.last_shots = (np.concatenate(kept_e) if kept_e else None, np.concatenate(kept_f) if kept_f else None)
        parallel.allreduce_counters(cnt)
        res = MCResult.from_words(cnt.cpu().numpy())
        self.last_result = res
        return res.failures, res.shots, int(sum(res.sector_nonconv))

    def _bposd_counts_host(self, num_run: int, batch: int = 16384, keep_shots: bool = False):
        """Host-assisted BP+OSD loop (non-uniform priors: the OSD half runs on the host stage)."""
        from .engine import DeviceMC, _torch

        torch = _torch()
        if self.seed is None:
            self.seed = random.getrandbits(64)
        need_x = self.eval_logical_type != "Z"
        need_z = self.eval_logical_type != "X"
        if getattr(self, "_bposd_mc", None) is None:
            self._bposd_mc = DeviceMC(self.code, self.decoder_x.decoder if need_x else None,
                                      self.decoder_z.decoder if need_z else None)
        mc = self._bposd_mc
        rank, ws = parallel.world()
        b, c = parallel.shard_range(num_run, rank, ws, begin=self._shot_offset)
        self._shot_offset += int(num_run)
        px, py, pz = self.channel_probs
        code = self.code
        sectors = [(0, need_x, self.decoder_x, code.csr("hz"), code.csr("lz")),
                   (1, need_z, self.decoder_z, code.csr("hx"), code.csr("lx"))]
        fails = osd_n = 0
        kept_e, kept_f = [], []
        dev = torch.device("cuda", mc.device)
        n = code.N
        for s0 in range(b, b + c, int(batch)):
            S = min(int(batch), b + c - s0)
            cnt = mc.new_counters()
            f_d = torch.zeros(S, dtype=torch.uint8, device=dev)
            e_d = torch.zeros((S, n), dtype=torch.uint8, device=dev)
            c_d = torch.zeros((S, 2, n), dtype=torch.uint8, device=dev)
            it_d = torch.zeros((S, 2), dtype=torch.int32, device=dev)
            mc.launch(px, py, pz, self.seed, s0, S, self.eval_logical_type, cnt, None, f_d, e_d, c_d, it_d)
            fail = f_d.cpu().numpy()
            sf = np.zeros((S, 2), dtype=bool)
            for q, need, dec, H, L in sectors:
                if not need:
                    continue
                f = ((fail >> q) & 1).astype(bool)
                # BP stopped before max_iter <=> it converged; only shots at max_iter may need OSD
                cand = torch.nonzero(it_d[:, q] >= dec.decoder.max_iter).flatten()
                if cand.numel():
                    ci = cand.cpu().numpy()
                    e = ((e_d[cand] >> q) & 1).cpu().numpy()
                    synd = gf2_rows(H, e)
                    bad = np.flatnonzero((gf2_rows(H, c_d[cand, q, :].cpu().numpy()) != synd).any(1))
                    if bad.size:
                        r = e[bad] ^ dec.decode_batch(synd[bad]).astype(np.uint8)
                        f[ci[bad]] = gf2_rows(H, r).any(1) | gf2_rows(L, r).any(1)
                        osd_n += int(bad.size)
                sf[:, q] = f
            if self.eval_logical_type == "X":
                fails += int(sf[:, 0].sum())
            elif self.eval_logical_type == "Z":
                fails += int(sf[:, 1].sum())
            else:
                fails += int((sf[:, 0] | sf[:, 1]).sum())
            if keep_shots:
                kept_e.append(e_d.cpu().numpy())
                kept_f.append(sf)
        if keep_shots:
            self.last_shots = (np.concatenate(kept_e) if kept_e else None, np.concatenate(kept_f) if kept_f else None)
        cnt = torch.tensor([fails, c, osd_n], dtype=torch.int64,
                           device=torch.device("cuda", mc.device))
        parallel.allreduce_counters(cnt)
        out = cnt.cpu().numpy()
        return int(out[0]), int(out[1]), int(out[2])

    def _batch_failures(self, n: int) -> int:
        ok, _, _ = self._engine_ready()
        if ok:
            return self.fused_counts(n).failures
        if self._bposd_ready():
            return self.bposd_counts(n)[0]
        return int(np.sum([self._single_run() for _ in range(n)]))

    def WordErrorRate(self, num_run: int):
        return word_error_rate(self._batch_failures(num_run), num_run, self.K)

    def WordErrorRate_TargetFailure(self, target_failures: int, batch_size: int, max_batches: int):
        """Adaptive sampling (the reference's ``WordErrorRate_TargetFailure``,
        src/Simulators_SpaceTime.py:1051-1077): batches of ``batch_size`` shots until
        ``target_failures`` failures or ``max_batches``; returns ``(wer, total_samples)``.
        Each batch's count is all-reduced, so every rank stops at the same batch."""
        total, fails = 0, 0
        for _ in range(int(max_batches)):
            fails += self._batch_failures(batch_size)
            total += int(batch_size)
            if fails >= target_failures:
                break
        return word_error_rate(fails, total, self.K)[0], total


def word_error_rate_phenl(error_count: int, num_samples: int, K: int, num_rounds: int):
    """``CodeSimulator_Phenon.WordErrorRate`` arithmetic (``src/Simulators.py:329-358``)."""
    assert int(num_rounds) % 2 == 1
    ler = error_count / num_samples
    ler_q = 1.0 - (1 - ler) ** (1 / K)
    if ler_q <= 0.5:
        return (1.0 - (1 - 2 * ler_q) ** (1 / num_rounds)) / 2
    return (1.0 + (-1 + 2 * ler_q) ** (1 / num_rounds)) / 2


class CodeSimulator_Phenon:
    """Single-shot phenomenological simulator (``src/Simulators.py:189-381``).

    Each noisy round decodes the extended syndrome ``[h | I]·[e | s_err]`` with
    decoder1 (``BP_Decoder_Class`` with ``p_syndrome``, or ``FirstMinBPDecoder``
    in the notebooks), then a perfect round is decoded by decoder2.  This is the
    space-time loop with ``num_rep = 1`` (``GetSpaceTimeCheckMat(h, 1) = [h | I]``,
    same draw order), so when decoder1_* are engine :class:`~.decoders.BPDecoder`
    objects on ``[h | I]`` and decoder2_* engine ``BPDecoder`` objects, every
    sample runs on the GPU (``qldpc_phenl_launch``).  Other decoders (e.g.
    ``FirstMinBPDecoder``) run the reference's per-sample loop.
    """

    def __init__(self, code=None, decoder1_x=None, decoder1_z=None, decoder2_x=None, decoder2_z=None,
                 pauli_error_probs=(0.01, 0.01, 0.01), q=0, eval_logical_type="Total", seed=None, max_batch=0):
        self.code = code
        self.hx_ext = np.hstack([code.hx, np.identity(np.shape(code.hx)[0])])
        self.hz_ext = np.hstack([code.hz, np.identity(np.shape(code.hz)[0])])
        self.decoder1_z, self.decoder1_x = decoder1_z, decoder1_x
        self.decoder2_z, self.decoder2_x = decoder2_z, decoder2_x
        self.N = code.N
        self.K = code.K
        self.channel_probs = list(pauli_error_probs)
        self.synd_prob = q
        self.error_x = np.zeros(self.N).astype(int)
        self.error_z = np.zeros(self.N).astype(int)
        self.min_logical_weight = self.N
        self.eval_logical_type = eval_logical_type
        self.seed = int(seed) if seed is not None else None
        self.max_batch = int(max_batch)
        self._shot_offset = 0
        self._ph = None
        self.last_result = None

    def _generate_error(self):
        """``:211-250``: data error (3-way split), then hx-row and hz-row syndrome flips."""
        N = self.N
        u = np.array([random.random() for _ in range(N)])
        ex, ez = pauli_split(u, self.channel_probs)
        sz = np.array([random.random() < self.synd_prob for _ in range(self.hx_ext.shape[1] - N)], dtype=int)
        sx = np.array([random.random() < self.synd_prob for _ in range(self.hz_ext.shape[1] - N)], dtype=int)
        self.error_x_ext = np.concatenate([ex, sx])
        self.error_z_ext = np.concatenate([ez, sz])
        return self.error_x_ext, self.error_z_ext

    def _single_run(self, num_rounds):
        """``:252-327``."""
        code = self.code
        N = self.N
        mx, mz = code.hx.shape[0], code.hz.shape[0]
        cz = np.zeros(N + mx, dtype=int)
        cx = np.zeros(N + mz, dtype=int)
        for _ in range(num_rounds - 1):
            ex_ext, ez_ext = self._generate_error()
            cx = (np.concatenate([cx[:N], np.zeros(mz, dtype=int)]) + ex_ext) % 2
            cz = (np.concatenate([cz[:N], np.zeros(mx, dtype=int)]) + ez_ext) % 2
            dz = np.asarray(self.decoder1_z.decode((self.hx_ext @ cz % 2).astype(int)))
            dx = np.asarray(self.decoder1_x.decode((self.hz_ext @ cx % 2).astype(int)))
            cx = (cx + dx.astype(int)) % 2
            cz = (cz + dz.astype(int)) % 2
        ex_ext, ez_ext = self._generate_error()
        cur_x = ((cx + ex_ext) % 2)[:N]
        cur_z = ((cz + ez_ext) % 2)[:N]
        dz = self.decoder2_z.decode(code.hx @ cur_z % 2)
        dx = self.decoder2_x.decode(code.hz @ cur_x % 2)
        rx, rz = (cur_x + dx) % 2, (cur_z + dz) % 2
        X_failure = int(((code.hz @ rx) % 2).any() or ((code.lz @ rx) % 2).any())
        Z_failure = int(((code.hx @ rz) % 2).any() or ((code.lx @ rz) % 2).any())
        assert self.eval_logical_type in ["X", "Z", "Total"]
        if self.eval_logical_type == "X":
            return X_failure
        if self.eval_logical_type == "Z":
            return Z_failure
        return X_failure or Z_failure

    def _engine_parts(self):
        from .decoders import BPDecoder

        d1 = (self.decoder1_x, self.decoder1_z)
        fm = self._firstmin1()
        if fm is None and not all(isinstance(d, BPDecoder) for d in d1):
            return None
        # decoder2 = engine BPDecoder, or BPOSD_Decoder with GPU OSD (the Threshold notebook's
        # BPDecoder + BPOSD_Decoder osd_e(10) pair): its soft BP feeds qldpc_phenl_set_final_osd
        b2 = tuple(_final_round_bp(d) for d in (self.decoder2_x, self.decoder2_z))
        if any(b is None for b in b2):
            return None
        if fm is not None:  # the pipeline's ST slot: a BP handle on the first-min decoders' own graphs
            return fm[0].st_bp(), fm[1].st_bp(), b2[0], b2[1]
        return d1[0].decoder, d1[1].decoder, b2[0], b2[1]

    def _firstmin1(self):
        """decoder1_x / decoder1_z as device first-min handles (FirstMinBPDecoder, minimum_sum, on
        [h | I] of this code: the Single-Shot notebook's decoder1), or None."""
        from .decoders import FirstMinBPDecoder

        d1 = (self.decoder1_x, self.decoder1_z)
        if not all(isinstance(d, FirstMinBPDecoder) and d._fm is not None for d in d1):
            return None
        ext = (self.hz_ext, self.hx_ext)
        if any(d.h.shape != e.shape or not np.array_equal(d.h % 2, e % 2) for d, e in zip(d1, ext)):
            return None
        return d1

    def _final_osd(self):
        return tuple(getattr(d, "gpu_osd", None) for d in (self.decoder2_x, self.decoder2_z))

    def fused_counts(self, num_rounds: int, num_samples: int):
        parts = self._engine_parts()
        if parts is None:
            raise TypeError("fused path needs engine BPDecoder instances (decoder1 on [h | I], decoder2 on h)")
        from .engine import DevicePhenl, MCResult, _torch

        torch = _torch()
        if self.seed is None:
            self.seed = random.getrandbits(64)
        if self._ph is None:
            self._ph = DevicePhenl(self.code, *parts, num_rep=1, max_batch=self.max_batch)
            ox, oz = self._final_osd()
            if ox is not None or oz is not None:
                self._ph.set_final_osd(ox, oz)
            fm = self._firstmin1()
            if fm is not None:
                self._ph.set_round_firstmin(fm[0]._fm, fm[1]._fm)
        rank, ws = parallel.world()
        b, c = parallel.shard_range(num_samples, rank, ws, begin=self._shot_offset)
        self._shot_offset += int(num_samples)
        px, py, pz = self.channel_probs
        cnt = self._ph.new_counters()
        self._ph.launch(px, py, pz, self.synd_prob, self.seed, b, c, num_rounds, self.eval_logical_type, cnt)
        parallel.allreduce_counters(cnt)
        torch.cuda.synchronize(cnt.device)
        res = MCResult.from_words(cnt.cpu().numpy())
        self.last_result = res
        return res

    def _count(self, num_rounds, num_samples):
        if self._engine_parts() is not None:
            return self.fused_counts(num_rounds, num_samples).failures
        return int(np.sum([self._single_run(num_rounds) for _ in range(num_samples)]))

    def WordErrorRate(self, num_rounds: int, num_samples: int):
        error_count = self._count(num_rounds, num_samples)
        return word_error_rate_phenl(error_count, num_samples, self.K, num_rounds), None

    def WordErrorProbability(self, num_rounds: int, num_samples: int):
        """``:360-381`` (the A8 formulas on the end-of-run failure count)."""
        return word_error_rate(self._count(num_rounds, num_samples), num_samples, self.K)


class CodeSimulator_Phenon_SpaceTime:
    """Phenomenological space-time simulator (``src/Simulators_SpaceTime.py:382-548``).

    ``WordErrorRate(num_cycles, num_samples)`` returns ``(wer, None)`` with the
    reference's per-cycle formula.  When decoder1_* are this engine's
    :class:`~.decoders.ST_BP_Decoder_syndrome` and decoder2_* its
    :class:`~.decoders.BPDecoder`, all samples run on the GPU
    (``qldpc_phenl_launch``: bit-sliced ballot sampling and syndromes, batched
    space-time BP, fold, final round, failure check), sharded over the
    ``torch.distributed`` ranks with one counter all-reduce.  Other decoders run
    the reference's per-sample ``_single_run`` loop.
    """

    def __init__(self, code=None, decoder1_x=None, decoder1_z=None, decoder2_x=None, decoder2_z=None,
                 pauli_error_probs=(0.01, 0.01, 0.01), q=0, eval_logical_type="Total", num_rep=1, seed=None,
                 max_batch=0):
        self.code = code
        self.hx_ext = np.hstack([code.hx, np.identity(np.shape(code.hx)[0])])
        self.hz_ext = np.hstack([code.hz, np.identity(np.shape(code.hz)[0])])
        self.decoder1_z, self.decoder1_x = decoder1_z, decoder1_x
        self.decoder2_z, self.decoder2_x = decoder2_z, decoder2_x
        self.N = code.N
        self.K = code.K
        self.channel_probs = list(pauli_error_probs)
        self.synd_prob = q
        self.min_logical_weight = self.N
        self.eval_logical_type = eval_logical_type
        self.num_rep = num_rep
        self.seed = int(seed) if seed is not None else None
        self.max_batch = int(max_batch)
        self._shot_offset = 0
        self._ph = None
        self.last_result = None

    # -- reference per-sample API (plugin path) --------------------------------
    def _generate_error(self):
        """``:405-442``: data error (3-way split), then hx-row and hz-row syndrome flips."""
        N = self.N
        u = np.array([random.random() for _ in range(N)])
        ex, ez = pauli_split(u, self.channel_probs)
        sz = np.array([random.random() < self.synd_prob for _ in range(self.hx_ext.shape[1] - N)], dtype=int)
        sx = np.array([random.random() < self.synd_prob for _ in range(self.hz_ext.shape[1] - N)], dtype=int)
        self.error_x_ext = np.concatenate([ex, sx])
        self.error_z_ext = np.concatenate([ez, sz])
        return self.error_x_ext, self.error_z_ext

    def _single_run(self, num_rounds):
        """``:444-529`` (Z detectors differenced, X raw: quirk Q3)."""
        code = self.code
        num_z_checks, num_qubits = code.hz.shape
        num_x_checks = code.hx.shape[0]
        cur_z, cur_x = np.zeros(num_qubits, dtype=int), np.zeros(num_qubits, dtype=int)
        for _ in range(num_rounds - 1):
            hist_z = np.zeros([self.num_rep, num_x_checks], dtype=int)
            hist_x = np.zeros([self.num_rep, num_z_checks], dtype=int)
            for j in range(self.num_rep):
                ex_ext, ez_ext = self._generate_error()
                cx = (np.concatenate([cur_x, np.zeros(num_z_checks, dtype=int)]) + ex_ext) % 2
                cz = (np.concatenate([cur_z, np.zeros(num_x_checks, dtype=int)]) + ez_ext) % 2
                hist_z[j] = (self.hx_ext @ cz % 2).astype(int)
                hist_x[j] = (self.hz_ext @ cx % 2).astype(int)
                cur_z, cur_x = cz[:num_qubits], cx[:num_qubits]
            det_z = hist_z.copy()
            det_z[1:] = (hist_z[:-1] + hist_z[1:]) % 2
            cur_z = (cur_z + self.decoder1_z.decode(det_z)) % 2
            cur_x = (cur_x + self.decoder1_x.decode(hist_x)) % 2
        ex_ext, ez_ext = self._generate_error()
        cur_x = (cur_x + ex_ext[:self.N]) % 2
        cur_z = (cur_z + ez_ext[:self.N]) % 2
        dz = self.decoder2_z.decode(code.hx @ cur_z % 2)
        dx = self.decoder2_x.decode(code.hz @ cur_x % 2)
        rx, rz = (cur_x + dx) % 2, (cur_z + dz) % 2
        X_failure = int(((code.hz @ rx) % 2).any() or ((code.lz @ rx) % 2).any())
        Z_failure = int(((code.hx @ rz) % 2).any() or ((code.lx @ rz) % 2).any())
        assert self.eval_logical_type in ["X", "Z", "Total"]
        if self.eval_logical_type == "X":
            return X_failure
        if self.eval_logical_type == "Z":
            return Z_failure
        return X_failure or Z_failure

    # -- fused engine path ----------------------------------------------------
    def _engine_parts(self):
        from .decoders import ST_BP_Decoder_syndrome

        d1 = (self.decoder1_x, self.decoder1_z)
        if not all(isinstance(d, ST_BP_Decoder_syndrome) and d.num_rep == self.num_rep for d in d1):
            return None
        b2 = tuple(_final_round_bp(d) for d in (self.decoder2_x, self.decoder2_z))
        if any(b is None for b in b2):
            return None
        return d1[0].space_decoder, d1[1].space_decoder, b2[0], b2[1]

    def _final_osd(self):
        return tuple(getattr(d, "gpu_osd", None) for d in (self.decoder2_x, self.decoder2_z))

    def fused_counts(self, num_rounds: int, num_samples: int):
        """Run ``num_samples`` samples on the GPU; returns the all-reduced :class:`~.engine.MCResult`."""
        parts = self._engine_parts()
        if parts is None:
            raise TypeError("fused path needs engine ST_BP_Decoder_syndrome (decoder1) and BPDecoder (decoder2)")
        from .engine import DevicePhenl, MCResult, _torch

        torch = _torch()
        if self.seed is None:
            self.seed = random.getrandbits(64)
        if self._ph is None:
            self._ph = DevicePhenl(self.code, *parts, num_rep=self.num_rep, max_batch=self.max_batch)
            ox, oz = self._final_osd()
            if ox is not None or oz is not None:
                self._ph.set_final_osd(ox, oz)
        rank, ws = parallel.world()
        b, c = parallel.shard_range(num_samples, rank, ws, begin=self._shot_offset)
        self._shot_offset += int(num_samples)
        px, py, pz = self.channel_probs
        cnt = self._ph.new_counters()
        self._ph.launch(px, py, pz, self.synd_prob, self.seed, b, c, num_rounds, self.eval_logical_type, cnt)
        parallel.allreduce_counters(cnt)
        torch.cuda.synchronize(cnt.device)
        res = MCResult.from_words(cnt.cpu().numpy())
        self.last_result = res
        return res

    def _batch_failures(self, num_rounds: int, n: int) -> int:
        if self._engine_parts() is not None:
            return self.fused_counts(num_rounds, n).failures
        return int(np.sum([self._single_run(num_rounds) for _ in range(n)]))

    def WordErrorRate(self, num_cycles: int, num_samples: int):
        num_rounds = int((num_cycles - 1) / self.num_rep + 1)
        error_count = self._batch_failures(num_rounds, num_samples)
        total_num_cycles = (num_rounds - 1) * self.num_rep + 1
        return word_error_rate_per_cycle(error_count, num_samples, self.K, total_num_cycles), None

    def WordErrorRate_TargetFailure(self, num_cycles: int, target_failures: int, batch_size: int, max_batches: int):
        """Adaptive sampling (src/Simulators_SpaceTime.py:1051-1077) on this simulator:
        batches until ``target_failures`` or ``max_batches``; returns ``(wer, total_samples)``."""
        num_rounds = int((num_cycles - 1) / self.num_rep + 1)
        total, fails = 0, 0
        for _ in range(int(max_batches)):
            fails += self._batch_failures(num_rounds, batch_size)
            total += int(batch_size)
            if fails >= target_failures:
                break
        total_num_cycles = (num_rounds - 1) * self.num_rep + 1
        return word_error_rate_per_cycle(fails, total, self.K, total_num_cycles), total


class CodeSimulator_Circuit_SpaceTime:
    """Circuit-level space-time simulator (``src/Simulators_SpaceTime.py:672-1077``).

    ``_generate_circuit`` builds the reference's syndrome-extraction circuits (:mod:`.circuit`:
    explicit op lists with stim's semantics, ``AddCXError`` noise) and the full circuit's detector
    error model; ``_generate_circuit_graph`` derives ``circuit_graph`` (h1 / L1 / channel_ps1 of
    the first layer, h2 / L2 / channel_ps2 of the last) and ``h1_space_cor`` from the one-round
    fault circuit's DEM, as ``GenFaultHyperGraph`` / ``GenCorrecHyperGraph`` do.  ``WordErrorRate``
    runs every sample on the GPU (``qldpc_circ_launch``: DEM mechanisms sampled by Philox,
    detectors by bit-sliced XOR, the round loop on the BP engine, decoder2 BP or BP+OSD) when
    decoder1_z / decoder2_z are this engine's decoders; other decoders run the reference's
    ``_decoding_samples`` loop per sample on GPU-sampled detectors.

    Deviation: for ``eval_logical_type='X'`` the reference swaps hx/hz and lx/lz IN the caller's
    code object (``:676-690``); here a shallow copy is swapped and the caller's object is left alone.
    """

    def __init__(self, code=None, decoder1_z=None, decoder1_x=None, decoder2_z=None, decoder2_x=None, p=0,
                 num_cycles=1, num_rep=1, error_params=None, eval_logical_type="Z", circuit_type="coloration",
                 rand_scheduling_seed=0, seed=None, max_batch=0, compat_dem_text=False, sampler="skip"):
        import copy as _copy

        from . import circuit as _circ

        if eval_logical_type == "X":  # :676-690, on a copy
            code = _copy.copy(code)
            code.hx, code.hz = code.hz, code.hx
            code.lx, code.lz = code.lz, code.lx
            decoder1_z, decoder2_z = decoder1_x, decoder2_x
        self.eval_code = code
        self.hx_ext = np.hstack([code.hx, np.identity(np.shape(code.hx)[0])])
        self.hz_ext = np.hstack([code.hz, np.identity(np.shape(code.hz)[0])])
        self.decoder1_z = decoder1_z
        self.decoder2_z = decoder2_z
        self.N = code.N
        self.K = code.K
        self.pz = p
        self.synd_prob = p
        self.min_logical_weight = self.N
        self.num_cycles = num_cycles
        self.num_rep = num_rep
        self.num_rounds = int((self.num_cycles - 1) / self.num_rep)
        assert np.abs((self.num_cycles - 1) / self.num_rep - self.num_rounds) <= 1e-2
        self.circuit = _circ.StimCircuit()
        self.fault_circuit = _circ.StimCircuit()
        self.error_params = error_params
        self.max_stab_weight_x = int(np.max(np.sum(code.hx, axis=1)))
        self.max_stab_weight_z = int(np.max(np.sum(code.hz, axis=1)))
        if circuit_type == "random":
            self.scheduling_X = _circ.RandomCircuit(code.hx)
            self.scheduling_Z = _circ.RandomCircuit(code.hz)
        elif circuit_type == "coloration":
            self.scheduling_X = _circ.ColorationCircuit(code.hx)
            self.scheduling_Z = _circ.ColorationCircuit(code.hz)
        self.num_logicals = self.eval_code.lx.shape[0]
        self.num_checks = self.eval_code.hx.shape[0]
        self.detector_sampler = None
        self.circuit_graph = None
        self.h1_space_cor = None
        self.dem = None
        self.fault_dem = None
        self.seed = int(seed) if seed is not None else None
        self.sampler = sampler  # DEM sampler of the device loop: "skip" (geometric gaps) or "keyed"
        self.max_batch = int(max_batch)
        self._shot_offset = 0
        self._dev = None
        self._dev_key = None
        self.last_result = None
        # True: the hypergraphs are built from the fault DEM rendered as stim's text and parsed with the
        # reference's regex (circuit.DetectorErrorModel.from_text): stim's mechanism order, 6-digit
        # probabilities, and mantissa-only reads of probabilities printed in exponent notation
        self.compat_dem_text = bool(compat_dem_text)

    # -- circuits and hypergraphs ---------------------------------------------------
    def _generate_circuit(self):
        """``:737-940``: the full circuit (num_rounds rounds + the final data measurement) and the
        one-round fault circuit, both with CX noise; the full circuit's DEM is the sampler."""
        from . import circuit as _circ

        c = self.eval_code
        self.circuit, self.fault_circuit = _circ.syndrome_circuits(
            c.hx, c.hz, c.lx, self.error_params, self.pz, self.num_rounds, self.num_rep, self.scheduling_X,
            self.scheduling_Z)
        self.dem = self.circuit.detector_error_model(flatten_loops=True)
        self.detector_sampler = _DetectorSampler(self)
        self._dev, self._dev_key = None, None  # a cached device loop holds the previous DEM

    def _generate_circuit_graph(self):
        """``:942-966``."""
        from . import circuit as _circ

        self.fault_dem = self.fault_circuit.detector_error_model(flatten_loops=True)
        src = self.fault_dem.to_text("stim") if self.compat_dem_text else self.fault_dem
        H_list, L_list, P_list = _circ.GenFaultHyperGraph(src, num_rounds=self.num_rounds,
                                                           num_rep=self.num_rep, num_logicals=self.num_logicals)
        self.circuit_graph = {"h1": H_list[0], "L1": L_list[0], "channel_ps1": P_list[0],
                              "h2": H_list[-1], "L2": L_list[-1], "channel_ps2": P_list[-1]}
        self.h1_space_cor = _circ.GenCorrecHyperGraph(src, num_rounds=self.num_rounds, num_rep=self.num_rep,
                                                      num_checks=self.num_checks, num_logicals=self.num_logicals)
        self._dev, self._dev_key = None, None  # new graphs: rebuild the device loop

    # -- reference per-sample path (plugin decoders) -------------------------------
    def _decoding_samples(self, samples):
        """``:968-1025``: per sample the round loop of decoder1, then decoder2; 1 = failure."""
        h1, L1 = self.circuit_graph["h1"], self.circuit_graph["L1"]
        h2, L2 = self.circuit_graph["h2"], self.circuit_graph["L2"]
        m, K = self.num_checks, len(self.eval_code.lx)
        out = []
        for sample in np.asarray(samples):
            hist = 1.0 * np.reshape(np.array(sample[:-K]), [self.num_cycles, m])
            logical = 1.0 * np.array(sample[-K:])
            dets = [np.reshape(hist[j * self.num_rep:(j + 1) * self.num_rep, :], [self.num_rep * m])
                    for j in range(self.num_rounds)]
            fin = hist[self.num_rounds * self.num_rep:, :]
            dets.append(np.reshape(fin, [fin.shape[0] * fin.shape[1]]))
            syn_cor, log_cor = 0, 0
            for j in range(self.num_rounds):
                syn = dets[j]
                syn[:m] = (syn[:m] + syn_cor) % 2
                cor = self.decoder1_z.decode(syn)
                syn_cor = (syn_cor + (self.h1_space_cor @ cor) % 2) % 2
                log_cor = (log_cor + L1 @ cor % 2) % 2
            final_syn = (dets[-1] + syn_cor) % 2
            final_cor = self.decoder2_z.decode(final_syn)
            log_cor = (log_cor + L2 @ final_cor % 2) % 2
            res_syn = (final_syn + h2 @ final_cor) % 2
            res_log = (logical + log_cor) % 2
            out.append(1 if (res_syn.any() or res_log.any()) else 0)
        return out

    def _single_run(self):
        samples = self.detector_sampler.sample(shots=1, append_observables=True)
        return self._decoding_samples(samples)[0]

    # -- fused engine path ---------------------------------------------------------
    def _engine_parts(self):
        """(decoder1's DeviceBP, decoder2's DeviceBP, decoder2's OSD or None), or None."""
        b1 = _engine_bp(self.decoder1_z)
        if b1 is None:
            return None
        d2 = self.decoder2_z
        if _is_bposd(d2):
            osd = getattr(d2, "gpu_osd", None) or d2.osd
            return b1, d2.decoder, osd
        b2 = _engine_bp(d2)
        return None if b2 is None else (b1, b2, None)

    def _device(self):
        from .engine import DeviceCircuit

        parts = self._engine_parts()
        key = None if parts is None else tuple(id(x) for x in parts)
        if self._dev is None or self._dev_key != key:
            if self.circuit_graph is None:
                raise RuntimeError("call _generate_circuit() and _generate_circuit_graph() first")
            cg = self.circuit_graph
            if parts is None:
                self._dev = DeviceCircuit(self.dem, max_batch=self.max_batch, sampler=self.sampler)
            else:
                b1, b2, osd = parts
                self._dev = DeviceCircuit(self.dem, b1, self.h1_space_cor, cg["L1"], b2, cg["L2"], self.num_rounds,
                                          self.num_rep, osd=osd, max_batch=self.max_batch, sampler=self.sampler)
            self._dev_key = key
        return self._dev

    def fused_counts(self, num_samples: int):
        """``num_samples`` samples on the GPU (sharded over the torch.distributed ranks); the
        all-reduced :class:`~.engine.MCResult`."""
        from .engine import MCResult, _torch

        if self._engine_parts() is None:
            raise TypeError("fused path needs engine decoders (ST_BP_Decoder_Circuit / BPDecoder / BPOSD_Decoder)")
        torch = _torch()
        if self.seed is None:
            self.seed = random.getrandbits(64)
        dev = self._device()
        rank, ws = parallel.world()
        b, c = parallel.shard_range(num_samples, rank, ws, begin=self._shot_offset)
        self._shot_offset += int(num_samples)
        cnt = dev.new_counters()
        dev.launch(self.seed, b, c, cnt)
        parallel.allreduce_counters(cnt)
        torch.cuda.synchronize(cnt.device)
        res = MCResult.from_words(cnt.cpu().numpy())
        self.last_result = res
        return res

    def _batch_failures(self, n: int) -> int:
        if self._engine_parts() is not None:
            return self.fused_counts(n).failures
        samples = self.detector_sampler.sample(shots=n, append_observables=True)
        return int(np.sum(self._decoding_samples(samples)))

    def WordErrorRate(self, num_samples: int):
        """``:1028-1049``: ``(wer per qubit per cycle, None)``; num_cycles must be odd."""
        error_count = self._batch_failures(num_samples)
        return word_error_rate_per_cycle(error_count, num_samples, self.K, self.num_cycles), None

    def WordErrorRate_TargetFailure(self, target_failures, batch_size, max_batches):
        """``:1051-1077``: batches until ``target_failures``; ``(wer, total_samples)``."""
        assert int(self.num_cycles) % 2 == 1
        total, fails = 0, 0
        for _ in range(int(max_batches)):
            fails += self._batch_failures(batch_size)
            total += int(batch_size)
            if fails >= target_failures:
                break
        print("failures:", fails)
        return word_error_rate_per_cycle(fails, total, self.K, self.num_cycles), total


class _DetectorSampler:
    """``self.circuit.compile_detector_sampler()`` (``:940``) on the GPU: the full circuit's DEM
    mechanisms sampled by Philox (``qldpc_circ_sample``); consecutive calls draw consecutive samples."""

    def __init__(self, sim: "CodeSimulator_Circuit_SpaceTime"):
        self.sim = sim

    def sample(self, shots: int, append_observables: bool = True):
        sim = self.sim
        if sim.seed is None:
            sim.seed = random.getrandbits(64)
        from .engine import DeviceCircuit

        dev = sim._dev if sim._dev is not None else DeviceCircuit(sim.dem, max_batch=sim.max_batch, sampler=sim.sampler)
        if sim._dev is None:
            sim._dev, sim._dev_key = dev, None
        out = dev.sample(sim.seed, sim._shot_offset, int(shots))
        sim._shot_offset += int(shots)
        return out if append_observables else out[:, :sim.dem.num_detectors]


# -------------------------------------------------------------- code family


class CodeFamily:
    """``src/Simulators.py:746-963`` (``'data'`` and ``'phenl'`` noise models; ``'circuit'`` needs stim)."""

    def __init__(self, code_list: list, decoder1_class, decoder2_class):
        self.code_list = code_list
        self.decoder1_class = decoder1_class
        self.decoder2_class = decoder2_class

    def EvalWER(self, noise_model: str, eval_logical_type: str, eval_p_list: list, num_samples: int, num_cycles=1,
                data_synd_noise_ratio=1, circuit_type="coloration", circuit_error_params=None, if_plot=True):
        assert noise_model in ["data", "phenl", "circuit"], "noise_model should be one of [data, phenl, circuit]"
        assert eval_logical_type in ["X", "Z", "Total"], "eval_type should be one of [X, Y, Total]"
        if noise_model == "circuit":
            raise NotImplementedError("circuit-level noise needs stim's circuits / detector error models (absent)")
        eval_wer_list = []
        for eval_code in self.code_list:
            for eval_p in eval_p_list:
                p = eval_p * 3 / 2
                pauli_error_probs = [p / 3, p / 3, p / 3]  # src/Simulators.py:763-764
                if noise_model == "phenl":  # src/Simulators.py:779-809
                    q = eval_p
                    p_data, p_synd = p * 2 / 3, q
                    hx_ext = np.hstack([eval_code.hx, np.identity(np.shape(eval_code.hx)[0])])
                    hz_ext = np.hstack([eval_code.hz, np.identity(np.shape(eval_code.hz)[0])])
                    d1x = self.decoder1_class.GetDecoder({"h": hz_ext, "p_data": p_data, "p_syndrome": p_synd})
                    d1z = self.decoder1_class.GetDecoder({"h": hx_ext, "p_data": p_data, "p_syndrome": p_synd})
                    d2x = self.decoder2_class.GetDecoder({"h": eval_code.hz, "p_data": p_data})
                    d2z = self.decoder2_class.GetDecoder({"h": eval_code.hx, "p_data": p_data})
                    sim = CodeSimulator_Phenon(code=eval_code, decoder1_x=d1x, decoder1_z=d1z, decoder2_x=d2x,
                                               decoder2_z=d2z, pauli_error_probs=pauli_error_probs, q=q,
                                               eval_logical_type=eval_logical_type)
                    eval_wer_list.append(sim.WordErrorRate(num_rounds=num_cycles, num_samples=num_samples)[0])
                    continue
                decoder_x = self.decoder2_class.GetDecoder({"h": eval_code.hz, "p_data": eval_p})
                decoder_z = self.decoder2_class.GetDecoder({"h": eval_code.hx, "p_data": eval_p})
                sim = CodeSimulator_DataError(code=eval_code, decoder_x=decoder_x, decoder_z=decoder_z,
                                              pauli_error_probs=pauli_error_probs,
                                              eval_logical_type=eval_logical_type)
                eval_wer_list.append(sim.WordErrorRate(num_samples)[0])
        eval_wer_array = np.reshape(np.array(eval_wer_list), [len(self.code_list), len(eval_p_list)])
        if if_plot:
            _plot_wer(self.code_list, eval_p_list, eval_wer_array, num_cycles)
        return eval_wer_array

    def EvalThreshold(self, noise_model: str, eval_logical_type: str, eval_method: str, est_threshold: float,
                      num_samples: int, num_cycles=1, data_synd_noise_ratio=1, circuit_type="coloration",
                      circuit_error_params=None, if_plot=False):
        """``src/Simulators.py:912-924``."""
        assert eval_method in ["extrapolation"], "eval_method should be one of [extrapolation]"
        eval_p_list = 10 ** (np.linspace(np.log10(est_threshold * 0.4), np.log10(est_threshold * 0.8), 6))
        eval_wer_array = self.EvalWER(noise_model, eval_logical_type, eval_p_list, num_samples, num_cycles,
                                      data_synd_noise_ratio, circuit_type, circuit_error_params, if_plot=False)
        return ThresholdEst_extrapolation(eval_p_list, eval_wer_array, if_plot)

    def EvalSustainableThreshold(self, noise_model: str, eval_logical_type: str, eval_method: str,
                                 est_threshold: float, num_samples_per_cycle: int, num_cycles_list: list,
                                 data_synd_noise_ratio=1, circuit_type="coloration", circuit_error_params=None,
                                 if_plot=False):
        """``src/Simulators.py:927-948``: the threshold at each cycle count (``num_samples_per_cycle /
        num_cycles`` samples each), then ``FitSusThreshold`` -> the sustainable threshold p_sus."""
        return _sustainable_threshold(self, noise_model, eval_logical_type, eval_method, est_threshold,
                                      num_samples_per_cycle, num_cycles_list, data_synd_noise_ratio, circuit_type,
                                      circuit_error_params, if_plot)

    def EvalEffectiveDistances(self, noise_model: str, eval_logical_type: str, eval_method: str, est_threshold: float,
                               num_samples: int, num_cycles=1, data_synd_noise_ratio=1, circuit_type="coloration",
                               if_plot=False):
        """``src/Simulators.py:951-963``: 5 log-spaced p in [p_th/6, p_th/4], then :func:`DistanceEst`."""
        assert noise_model in ["data", "phenl", "circuit"], "noise_model should be one of [data, phenl, circuit]"
        assert eval_logical_type in ["X", "Z", "Total"], "eval_type should be one of [X, Y, Total]"
        assert eval_method in ["extrapolation"], "eval_method should be one of [extrapolation]"
        eval_p_list = 10 ** (np.linspace(np.log10(est_threshold / 6), np.log10(est_threshold / 4), 5))
        eval_wer_array = self.EvalWER(noise_model, eval_logical_type, eval_p_list, num_samples, num_cycles,
                                      data_synd_noise_ratio, circuit_type, if_plot=False)
        return DistanceEst(eval_p_list, eval_wer_array, if_plot)


def FitSusThreshold(N, p_sus, p_0, gamma):
    """Sustainable-threshold model of ``EvalSustainableThreshold`` (``src/Simulators.py:936-938``)."""
    return p_sus * (1 - (1 - p_0 / p_sus) * np.exp(-gamma * N))


def _sustainable_threshold(fam, noise_model, eval_logical_type, eval_method, est_threshold, num_samples_per_cycle,
                           num_cycles_list, data_synd_noise_ratio, circuit_type, circuit_error_params, if_plot):
    from scipy.optimize import curve_fit

    sweep = [fam.EvalThreshold(noise_model=noise_model, eval_logical_type=eval_logical_type, eval_method=eval_method,
                               est_threshold=est_threshold, num_samples=int(num_samples_per_cycle / c), num_cycles=c,
                               data_synd_noise_ratio=data_synd_noise_ratio, circuit_type=circuit_type,
                               circuit_error_params=circuit_error_params, if_plot=if_plot) for c in num_cycles_list]
    popt, _ = curve_fit(FitSusThreshold, np.array(num_cycles_list), np.array(sweep), p0=(0.01, 0.05, 0.05))
    if if_plot:
        try:
            import matplotlib.pyplot as plt

            plt.figure()
            plt.plot(num_cycles_list, sweep, "D")
            plt.plot(num_cycles_list, FitSusThreshold(np.array(num_cycles_list), *popt), "-")
            plt.close()
        except ImportError:
            pass
    return popt[0]


class CodeFamily_SpaceTime:
    """``src/Simulators_SpaceTime.py:1152-1309`` for the ``'data'`` and ``'phenl'`` noise models.

    ``'phenl'`` builds decoder1 (space-time, ``num_rep``) and decoder2 exactly
    as the reference (``:1189-1216``; p_data = eval_p, q = eval_p, Pauli
    ``[eval_p/2]*3``) and runs :class:`CodeSimulator_Phenon_SpaceTime` (the
    reference names an undefined ``CodeSimulator_SpaceTime`` there, quirk Q5).
    Return shapes (``:1165-1296``): ``'data'`` — ``(eval_wer_list, eval_p_list)``, one ``np.array``
    of WERs per code and the p list exactly as passed, as the reference.  ``'phenl'`` — the
    reference appends one scalar per (code, p) to a flat list and then fails at its ``return`` on
    the unbound ``eval_p_adapt_list`` (UnboundLocalError); here it returns the same values
    nested like ``'data'`` (``eval_wer_list[c][i]`` = code c at ``eval_p_list[i]``, i.e. the
    reference's flat list reshaped to ``[len(code_list), len(eval_p_list)]`` as its commented-out
    ``np.reshape`` does) and one p array per code.  ``'circuit'`` (``:1220-1268``) builds the circuit
    and fault graphs per (code, p) with :class:`CodeSimulator_Circuit_SpaceTime` (stim's role restated
    in :mod:`.circuit`) and returns ``(eval_wer_list, eval_p_adapt_list)`` like the reference.
    """

    def __init__(self, code_list: list, decoder1_class, decoder2_class):
        self.code_list = code_list
        self.decoder1_class = decoder1_class
        self.decoder2_class = decoder2_class

    def EvalWER(self, noise_model: str, eval_logical_type: str, eval_p_list: list, num_samples: int, num_cycles=1,
                num_rep=1, circuit_type="coloration", circuit_error_params=None, if_plot=True, if_adaptive=False,
                adaptive_params=None):
        assert noise_model in ["data", "phenl", "circuit"], "noise_model should be one of [data, phenl, circuit]"
        assert eval_logical_type in ["X", "Z", "Total"], "eval_type should be one of [X, Y, Total]"
        if noise_model == "circuit":
            return self._eval_wer_circuit(eval_logical_type, eval_p_list, num_samples, num_cycles, num_rep,
                                          circuit_type, circuit_error_params, if_adaptive, adaptive_params)
        eval_wer_list, eval_p_adapt_list = [], []
        for eval_code in self.code_list:
            per_code = []
            for eval_p in eval_p_list:
                p = eval_p * 3 / 2
                pauli_error_probs = [p / 3, p / 3, p / 3]
                if noise_model == "data":
                    dx = self.decoder2_class.GetDecoder({"h": eval_code.hz, "p_data": eval_p})
                    dz = self.decoder2_class.GetDecoder({"h": eval_code.hx, "p_data": eval_p})
                    sim = CodeSimulator_DataError(code=eval_code, decoder_x=dx, decoder_z=dz,
                                                  pauli_error_probs=pauli_error_probs,
                                                  eval_logical_type=eval_logical_type)
                    per_code.append(sim.WordErrorRate(num_samples)[0])
                else:
                    q = eval_p
                    p_data, p_synd = p * 2 / 3, q
                    d1x = self.decoder1_class.GetDecoder({"h": eval_code.hz, "p_data": p_data, "p_syndrome": p_synd,
                                                          "num_rep": num_rep})
                    d1z = self.decoder1_class.GetDecoder({"h": eval_code.hx, "p_data": p_data, "p_syndrome": p_synd,
                                                          "num_rep": num_rep})
                    d2x = self.decoder2_class.GetDecoder({"h": eval_code.hz, "p_data": p_data})
                    d2z = self.decoder2_class.GetDecoder({"h": eval_code.hx, "p_data": p_data})
                    sim = CodeSimulator_Phenon_SpaceTime(code=eval_code, decoder1_x=d1x, decoder1_z=d1z,
                                                         decoder2_x=d2x, decoder2_z=d2z,
                                                         pauli_error_probs=pauli_error_probs, q=q,
                                                         eval_logical_type=eval_logical_type, num_rep=num_rep)
                    per_code.append(sim.WordErrorRate(num_cycles=num_cycles, num_samples=num_samples)[0])
            eval_wer_list.append(np.array(per_code))
            eval_p_adapt_list.append(np.array(eval_p_list))
        if noise_model == "data":
            return eval_wer_list, eval_p_list  # :1166 eval_p_adapt_list = eval_p_list
        return eval_wer_list, eval_p_adapt_list

    def _eval_wer_circuit(self, eval_logical_type, eval_p_list, num_samples, num_cycles, num_rep, circuit_type,
                          circuit_error_params, if_adaptive, adaptive_params):
        """``src/Simulators_SpaceTime.py:1220-1268``: per code the (optionally WEREst-pruned) p list;
        per p the circuit and fault graphs, decoder1 on h1 and decoder2 on h2 from the factories
        (``code_h`` = hx), then ``WordErrorRate(num_samples)``."""
        eval_wer_list, eval_p_adapt_list = [], []
        for eval_code in self.code_list:
            if if_adaptive:
                WEREst, min_wer = adaptive_params["WEREst"], adaptive_params["min_wer"]
                plist = [ep for ep in eval_p_list if WEREst(eval_code.N, ep) >= min_wer]
            else:
                plist = eval_p_list
            per_code = []
            for eval_p in plist:
                p = eval_p
                cep = circuit_error_params
                error_params = {k: cep[k] * p for k in ("p_i", "p_state_p", "p_m", "p_CX", "p_idling_gate")}
                sim = CodeSimulator_Circuit_SpaceTime(code=eval_code, decoder1_z=None, decoder1_x=None,
                                                      decoder2_z=None, decoder2_x=None, p=p, num_cycles=num_cycles,
                                                      num_rep=num_rep, error_params=error_params,
                                                      eval_logical_type=eval_logical_type, circuit_type=circuit_type,
                                                      rand_scheduling_seed=1)
                sim._generate_circuit()
                sim._generate_circuit_graph()
                g = sim.circuit_graph
                sim.decoder1_z = self.decoder1_class.GetDecoder({"code_h": eval_code.hx, "h": g["h1"],
                                                                 "channel_probs": g["channel_ps1"]})
                sim.decoder2_z = self.decoder2_class.GetDecoder({"code_h": eval_code.hx, "h": g["h2"],
                                                                 "channel_probs": g["channel_ps2"]})
                per_code.append(sim.WordErrorRate(num_samples=num_samples)[0])
            eval_p_adapt_list.append(np.array(plist))
            eval_wer_list.append(np.array(per_code))
        return eval_wer_list, eval_p_adapt_list

    def EvalThreshold(self, noise_model: str, eval_logical_type: str, eval_method: str, est_threshold: float,
                      num_samples: int, num_cycles=1, data_synd_noise_ratio=1, circuit_type="coloration",
                      circuit_error_params=None, if_plot=False):
        """``src/Simulators_SpaceTime.py:1311-1324``.  As in the reference, ``data_synd_noise_ratio`` is
        passed positionally into EvalWER's ``num_rep`` slot (quirk Q7); the WER list (first element of
        EvalWER's pair; the reference hands the pair itself to the fit, which cannot work) is fitted."""
        assert noise_model in ["data", "phenl", "circuit"], "noise_model should be one of [data, phenl, circuit]"
        assert eval_logical_type in ["X", "Z", "Total"], "eval_type should be one of [X, Y, Total]"
        assert eval_method in ["extrapolation"], "eval_method should be one of [extrapolation]"
        eval_p_list = 10 ** (np.linspace(np.log10(est_threshold * 0.4), np.log10(est_threshold * 0.8), 6))
        res = self.EvalWER(noise_model, eval_logical_type, eval_p_list, num_samples, num_cycles, data_synd_noise_ratio,
                           circuit_type, circuit_error_params, if_plot=False)
        wer = res[0] if isinstance(res, tuple) else res
        return ThresholdEst_extrapolation(eval_p_list, np.array(wer), if_plot)

    def EvalSustainableThreshold(self, noise_model: str, eval_logical_type: str, eval_method: str,
                                 est_threshold: float, num_samples_per_cycle: int, num_cycles_list: list,
                                 data_synd_noise_ratio=1, circuit_type="coloration", circuit_error_params=None,
                                 if_plot=False):
        """``src/Simulators_SpaceTime.py:1326-1347`` (same as CodeFamily's)."""
        return _sustainable_threshold(self, noise_model, eval_logical_type, eval_method, est_threshold,
                                      num_samples_per_cycle, num_cycles_list, data_synd_noise_ratio, circuit_type,
                                      circuit_error_params, if_plot)

    def EvalEffectiveDistances(self, noise_model: str, eval_logical_type: str, eval_method: str, est_threshold: float,
                               num_samples: int, num_cycles=1, data_synd_noise_ratio=1, circuit_type="coloration",
                               if_plot=False):
        """``src/Simulators_SpaceTime.py:1350-1362`` (``data_synd_noise_ratio`` lands in ``num_rep``, Q7)."""
        assert noise_model in ["data", "phenl", "circuit"], "noise_model should be one of [data, phenl, circuit]"
        assert eval_logical_type in ["X", "Z", "Total"], "eval_type should be one of [X, Y, Total]"
        assert eval_method in ["extrapolation"], "eval_method should be one of [extrapolation]"
        eval_p_list = 10 ** (np.linspace(np.log10(est_threshold / 6), np.log10(est_threshold / 4), 5))
        res = self.EvalWER(noise_model, eval_logical_type, eval_p_list, num_samples, num_cycles, data_synd_noise_ratio,
                           circuit_type, if_plot=False)
        wer = res[0] if isinstance(res, tuple) else res
        return DistanceEst(eval_p_list, np.array(wer), if_plot)


def _plot_wer(code_list, eval_p_list, eval_wer_array, num_cycles):
    try:
        import matplotlib.pyplot as plt
    except ImportError:  # plotting is cosmetic in the reference too
        return
    per_qubit = (1 - (1 - 2 * eval_wer_array) ** num_cycles) / 2
    total = np.zeros(eval_wer_array.shape)
    for i, code in enumerate(code_list):
        total[i, :] = 1 - (1 - per_qubit[i, :]) ** code.K
    fig, ax = plt.subplots(1, 3, figsize=(15, 3))
    for arr, a, lab in ((total, ax[0], "Logical error"), (per_qubit, ax[1], "Logical error per qubit"),
                        (eval_wer_array, ax[2], "WER")):
        for row in arr:
            a.plot(eval_p_list, row, "D--")
        a.set_xscale("log")
        a.set_yscale("log")
        a.set_xlabel(r"$p$")
        a.set_ylabel(lab)
    plt.close(fig)


# ------------------------------------------------------- threshold fitting


def CriticalExponentFit(xdata_tuple, pc, nu, A, B, C):
    """``src/Simulators.py:674-678`` (unused by the reference's estimators; kept for the API)."""
    p, d = xdata_tuple
    x = (p - pc) * d ** (1 / nu)
    return A + B * x + C * x ** 2


def EmpericalFit(xdata_tuple, pc, A):
    p, d = xdata_tuple
    return A * (p / pc) ** (d / 2)


def FitDistance(p, A, d):
    return A * p ** (d / 2)


def DistanceEst(sweep_p_list, sweep_pl_total_list, if_plot=False):
    """``src/Simulators.py:690-699``."""
    from scipy.optimize import curve_fit

    out = []
    for sweep_pl_list in sweep_pl_total_list:
        popt, _ = curve_fit(FitDistance, np.array(sweep_p_list), np.array(sweep_pl_list) + 1e-10, p0=(0.01, 3))
        out.append(popt[1])
    return out


def ThresholdEst_extrapolation(sweep_p_list, sweep_pl_total_list, if_plot=False):
    """``src/Simulators.py:701-741`` (fit ``A (p/p_c)^(d/2)`` with per-code fitted d)."""
    from scipy.optimize import curve_fit

    num_p = len(sweep_p_list)
    num_code = len(sweep_pl_total_list)
    d_list = DistanceEst(sweep_p_list, sweep_pl_total_list)
    p_all = list(sweep_p_list) * num_code
    d_all = [d for d in d_list for _ in range(num_p)]
    fit_X = np.vstack([np.reshape(np.array(p_all), [1, num_p * num_code]),
                       np.reshape(np.array(d_all), [1, num_p * num_code])])
    fit_Z = np.reshape(np.array(sweep_pl_total_list), [num_p * num_code])
    popt, _ = curve_fit(EmpericalFit, fit_X, fit_Z, p0=(0.04, 0.1))
    print("p_c:", popt[0])
    return popt[0]
