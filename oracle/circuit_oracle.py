"""CPU oracle for the circuit-level space-time path (TEST INFRASTRUCTURE ONLY: imported by tests/,
never by the product package).

Two independent restatements the product (``qldpc_fault_tolerance_amd/circuit.py`` and the HIP
pipeline ``csrc/circuit.hip``) is checked against:

* :func:`dem_forward` — the detector error model by FORWARD Pauli-frame propagation, one fault at a
  time: every Pauli component of every noise instruction is injected at its location and pushed
  through the rest of the circuit (H swaps x/z; CX c->t: x_t ^= x_c, z_c ^= z_t; Z-basis measurement
  flips on x, X-basis on z; resets clear the frame), the flipped measurement records give the
  symptom.  The product's analysis runs BACKWARDS with per-qubit sensitivity bitsets; identical
  symptom -> probability maps are the check.  Stim's channel decompositions
  (``src/Simulators_SpaceTime.py:950`` calls ``detector_error_model``) are restated in both.
* :func:`circuit_run` — ``CodeSimulator_Circuit_SpaceTime`` per sample
  (``src/Simulators_SpaceTime.py:968-1025``): sample every DEM mechanism of the full circuit
  (Philox uniform of (seed, shot, mechanism) in the circuit stream < p), detectors / observables as
  XORs, then ``_decoding_samples``' round loop with the oracle's BP (decoder1 on h1) and BP+OSD
  (decoder2 on h2), exactly the reference's arithmetic order.
"""
from __future__ import annotations

import math

import numpy as np

import oracle

STREAM_CIRC = 0x51D50003  # Philox counter word 3 of the circuit-level mechanism stream


def _d1(p):
    return 0.5 - 0.5 * math.sqrt(1.0 - (4.0 * p) / 3.0)


def _d2(p):
    return 0.5 - 0.5 * (1.0 - (16.0 * p) / 15.0) ** 0.125


def dem_forward(circuit):
    """{(dets tuple, obs tuple): probability} by forward propagation of each fault."""
    ops = circuit.ops
    nq = max(circuit.num_qubits, 1)
    # records and detector / observable definitions
    nrec, recbase, dets, obs = 0, [], [], {}
    for o in ops:
        recbase.append(nrec)
        if o.name in ("M", "MR", "MX"):
            nrec += len(o.targets)
        elif o.name == "DETECTOR":
            dets.append([nrec + k for k in o.targets])
        elif o.name == "OBSERVABLE_INCLUDE":
            obs.setdefault(int(o.arg), []).extend(nrec + k for k in o.targets)

    def propagate(t0, frame_x, frame_z):
        x, z = dict(frame_x), dict(frame_z)
        flips = set()
        for t in range(t0 + 1, len(ops)):
            o = ops[t]
            nm, tg = o.name, o.targets
            if nm == "H":
                for q in tg:
                    x[q], z[q] = z.get(q, 0), x.get(q, 0)
            elif nm == "CX":
                for i in range(0, len(tg), 2):
                    c, u = tg[i], tg[i + 1]
                    x[u] = x.get(u, 0) ^ x.get(c, 0)
                    z[c] = z.get(c, 0) ^ z.get(u, 0)
            elif nm in ("R", "RX"):
                for q in tg:
                    x[q] = z[q] = 0
            elif nm in ("M", "MR", "MX"):
                for i, q in enumerate(tg):
                    f = x.get(q, 0) if nm != "MX" else z.get(q, 0)
                    if f:
                        flips.add(recbase[t] + i)
                    if nm == "MR":
                        x[q] = z[q] = 0
        d = tuple(i for i, rs in enumerate(dets) if sum(r in flips for r in rs) % 2)
        k = tuple(i for i in sorted(obs) if sum(r in flips for r in obs[i]) % 2)
        return d, k

    out = {}

    def add(sym, p):
        if (not sym[0] and not sym[1]) or p <= 0:
            return
        if sym in out:
            q = out[sym]
            out[sym] = q * (1 - p) + p * (1 - q)
        else:
            out[sym] = p

    paulis1 = [(1, 0), (1, 1), (0, 1)]  # X, Y, Z as (x, z)
    for t, o in enumerate(ops):
        if o.name == "DEPOLARIZE1" and o.arg > 0:
            pc = _d1(o.arg)
            for q in o.targets:
                for px, pz in paulis1:
                    add(propagate(t, {q: px}, {q: pz}), pc)
        elif o.name == "DEPOLARIZE2" and o.arg > 0:
            pc = _d2(o.arg)
            tg = o.targets
            for i in range(0, len(tg), 2):
                a, b = tg[i], tg[i + 1]
                for pa in range(4):
                    for pb in range(4):
                        if pa == 0 and pb == 0:
                            continue
                        fx = {a: pa in (1, 2), b: pb in (1, 2)}
                        fz = {a: pa in (2, 3), b: pb in (2, 3)}
                        if a == b:
                            raise ValueError("DEPOLARIZE2 on a repeated qubit")
                        add(propagate(t, {k: int(v) for k, v in fx.items()}, {k: int(v) for k, v in fz.items()}), pc)
        elif o.name == "X_ERROR" and o.arg > 0:
            for q in o.targets:
                add(propagate(t, {q: 1}, {}), o.arg)
        elif o.name == "Z_ERROR" and o.arg > 0:
            for q in o.targets:
                add(propagate(t, {}, {q: 1}), o.arg)
    return out


def dem_as_map(dem):
    return {(tuple(d), tuple(k)): p for p, d, k in zip(dem.probs, dem.dets, dem.obs)}


def sample_mechanisms_keyed(probs, seed, shot_begin, shot_count):
    """[S][M] uint8, the keyed sampler (``qldpc_circ_set_sampler(c, 0)``): mechanism j of shot s fires
    when Philox uniform(seed, shot, j) < p_j."""
    M = len(probs)
    out = np.zeros((shot_count, M), np.uint8)
    for s in range(shot_count):
        for j, p in enumerate(probs):
            out[s, j] = oracle.uniform(seed, shot_begin + s, j, STREAM_CIRC) < p
    return out


STREAM_SKIP = 0x51D50004  # Philox counter word 3 of the geometric-skip sampler (csrc/circuit.hip kStreamSkip)


def _ceil53(t):
    return math.ceil(math.ldexp(t, 53)) if t > 0.0 else 0


def skip_thresholds(p):
    """T_k = ceil(2^53 (1 - p)^k), k = 1..64, (1 - p)^k by repeated IEEE multiplication (as the
    library's host table in qldpc_circ_create)."""
    q, t, out = 1.0 - float(p), 1.0, []
    for _ in range(64):
        t *= q
        out.append(_ceil53(t))
    return out


def skip_word(seed, j, gw, T):
    """The 64 samples 64 gw .. 64 gw + 63 of mechanism j as a bit word (bit b = sample 64 gw + b):
    from position pos, G = #{k in 1..64-pos : u < T_k} non-firing samples, then a firing; u the 53-bit
    Philox integer of (seed, j, gw, draw index c) (csrc/circuit.hip skip_word)."""
    bits, pos, c = 0, 0, 0
    while c <= 64:
        shot = (gw & 0xFFFFFFFF) | ((((gw >> 32) << 8) | c) << 32)
        u = int(oracle.uniform(seed, shot, j, STREAM_SKIP) * 9007199254740992.0)
        g = 0
        while g < 64 - pos and T[g] > u:  # T non-increasing: the count of k with T_k > u
            g += 1
        pos += g
        if pos >= 64:
            break
        bits |= 1 << pos
        pos += 1
        c += 1
    return bits


def sample_mechanisms(probs, seed, shot_begin, shot_count):
    """[S][M] uint8, the geometric-skip sampler (the default, ``qldpc_circ_set_sampler(c, 1)``):
    per mechanism the global 64-sample words covering the shots, each from :func:`skip_word`."""
    M = len(probs)
    out = np.zeros((shot_count, M), np.uint8)
    if shot_count <= 0:
        return out
    g0, g1 = shot_begin >> 6, (shot_begin + shot_count - 1) >> 6
    for j, p in enumerate(probs):
        T = skip_thresholds(p)
        for gw in range(g0, g1 + 1):
            w = skip_word(seed, j, gw, T)
            while w:
                b = (w & -w).bit_length() - 1
                w &= w - 1
                s = gw * 64 + b - shot_begin
                if 0 <= s < shot_count:
                    out[s, j] = 1
    return out


def circuit_run(dem_full, h1, L1, p1, h1_space_cor, h2, L2, p2, num_rounds, num_rep, m, max_iter1, max_iter2,
                seed, shot_begin, shot_count, osd_method="osd_e", osd_order=10, ms_scaling_factor=0.625,
                precision=64, final_osd=True):
    """Per-sample failure flags of ``CodeSimulator_Circuit_SpaceTime`` (see the module docstring)."""
    H = dem_full.check_matrix().astype(np.int64)
    Lf = dem_full.observable_matrix().astype(np.int64)
    e = sample_mechanisms(dem_full.probs, seed, shot_begin, shot_count).astype(np.int64)
    det = (e @ H.T) % 2
    logical = (e @ Lf.T) % 2
    K = Lf.shape[0]
    h1 = np.asarray(h1, np.uint8)
    h2 = np.asarray(h2, np.uint8)
    hs = np.asarray(h1_space_cor, np.int64)
    L1 = np.asarray(L1, np.int64)
    L2 = np.asarray(L2, np.int64)
    S = shot_count
    acc_syn = np.zeros((S, m), np.int64)
    acc_log = np.zeros((S, K), np.int64)
    R1 = num_rep * m
    for j in range(num_rounds):
        syn = det[:, j * R1:(j + 1) * R1].copy()
        syn[:, :m] = (syn[:, :m] + acc_syn) % 2
        cor, _, _ = oracle.bp_decode_batch(h1, np.asarray(p1), max_iter1, "minimum_sum", ms_scaling_factor,
                                           syn.astype(np.uint8), precision)
        cor = cor.astype(np.int64)
        acc_syn = (acc_syn + cor @ hs.T) % 2
        acc_log = (acc_log + cor @ L1.T) % 2
    fin = (det[:, num_rounds * R1:num_rounds * R1 + m] + acc_syn) % 2
    if final_osd:
        bp, _, conv, post = oracle.bp_decode_batch_soft(h2, np.asarray(p2), max_iter2, ms_scaling_factor,
                                                        fin.astype(np.uint8), precision)
        _, osdw = oracle.osd_decode_batch(h2, np.asarray(p2), fin.astype(np.uint8), post, osd_method, osd_order)
        cor2 = np.where(conv[:, None].astype(bool), bp, osdw).astype(np.int64)
    else:
        cor2, _, _ = oracle.bp_decode_batch(h2, np.asarray(p2), max_iter2, "minimum_sum", ms_scaling_factor,
                                            fin.astype(np.uint8), precision)
        cor2 = cor2.astype(np.int64)
    res_syn = (fin + cor2 @ h2.astype(np.int64).T) % 2
    res_log = (logical + acc_log + cor2 @ L2.T) % 2
    fail = (res_syn.any(axis=1) | res_log.any(axis=1)).astype(np.uint8)
    return {"fail": fail, "failures": int(fail.sum()), "det": det.astype(np.uint8), "logical": logical.astype(np.uint8)}
