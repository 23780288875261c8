"""Circuit-level space-time noise: stabilizer circuits, their detector error
models (DEMs) and the fault hypergraphs the reference decodes on.

The reference builds its syndrome-extraction circuit with ``stim`` op by op
(``CodeSimulator_Circuit_SpaceTime._generate_circuit``, ``src/Simulators_SpaceTime.py:737-940``),
inserts two-qubit gate noise by rewriting the circuit text (``AddCXError``,
``src/ErrorPlugin.py:11-25``), asks stim for the detector error model
(``detector_error_model(flatten_loops=True)``, ``:950, :963``) and parses its text into the decoding
hypergraphs (``GenFaultHyperGraph`` / ``GenCorrecHyperGraph``, ``:551-668``).  stim is absent here
(and not installable), so this module restates, from scratch:

* :class:`StimCircuit` — an explicit op list with stim's append semantics (consecutive appends of
  the same gate and argument fuse into one instruction, ``+`` concatenates, ``n * c`` repeats);
* :func:`add_cx_error` — ``AddCXError``: a ``DEPOLARIZE2(p)`` on the same target pairs right after
  every ``CX`` instruction;
* :func:`detector_error_model` — a Pauli-frame analysis, run backwards over the flattened circuit:
  per qubit the sets of detectors / observables an X or a Z error at that point flips (bitsets),
  so every fault's symptom is one XOR.  Depolarizing channels are split into independent Pauli
  mechanisms with stim's per-channel probabilities (``DEPOLARIZE1(p)``: X, Y, Z each with
  ``(1 - sqrt(1 - 4p/3)) / 2``; ``DEPOLARIZE2(p)``: the 15 non-identity two-qubit Paulis each with
  ``(1 - (1 - 16p/15)^(1/8)) / 2``), which reproduces the channel's distribution exactly; mechanisms
  with identical symptoms merge (``p1 (1 - p2) + p2 (1 - p1)``), empty symptoms drop;
* :func:`GenFaultHyperGraph` / :func:`GenCorrecHyperGraph` on that DEM, with the reference's layer
  logic (first and last ``shift_detectors`` segments);
* :func:`ColorationCircuit` / :func:`RandomCircuit` — the CX schedules of
  ``src/CircuitScheduling.py:73-131`` (networkx's Hopcroft-Karp matching, the dependency the
  reference itself calls, on the same graph built in the same order).

Parity: the schedules are pinned against the reference's own ``CircuitScheduling`` (importable
here: numpy + networkx), ``tests/golden/reference_circuit_schedules.npz``.  The DEM is checked
against an independent forward-propagation restatement (``oracle/circuit_oracle.py``) and
hand-derived DEMs of small circuits; against stim itself it is **parity unpinned** (stim's DEM
mechanism order, and the text the reference parses with ``re.findall("\\d+\\.\\d+", ...)``, are not
reproduced: probabilities stay exact doubles).  The only stim-era output the reference holds is
the demo's WER 1.93e-4 (``SpaceTimeDecodingDemo.ipynb`` cell 3), checked statistically on the GPU.
"""
from __future__ import annotations

import copy
import math
import random
from dataclasses import dataclass, field

import numpy as np

# gates the analysis understands; annotations carry no Pauli-frame action
_FUSABLE = {"R", "RX", "H", "CX", "M", "MR", "MX", "DEPOLARIZE1", "DEPOLARIZE2", "X_ERROR", "Z_ERROR"}
_ANNOT = {"DETECTOR", "OBSERVABLE_INCLUDE", "SHIFT_COORDS", "TICK"}


@dataclass
class Op:
    name: str
    targets: list
    arg: float | None = None


class StimCircuit:
    """An explicit, flattened stim-style op list.  ``DETECTOR`` / ``OBSERVABLE_INCLUDE`` targets are
    negative measurement-record offsets (``stim.target_rec(k)``)."""

    def __init__(self, ops=None):
        self.ops: list[Op] = [Op(o.name, list(o.targets), o.arg) for o in (ops or [])]

    def append(self, name: str, targets=(), arg=None):
        name = name.upper()
        if name not in _FUSABLE and name not in _ANNOT:
            raise ValueError(f"gate {name!r} is not supported by this circuit model")
        targets = [int(t) for t in np.asarray(targets, dtype=np.int64).reshape(-1)] if len(targets) else []
        if isinstance(arg, (list, tuple)):
            arg = float(arg[0]) if len(arg) else None
        arg = None if arg is None else float(arg)
        last = self.ops[-1] if self.ops else None
        # stim fuses an append into the previous instruction when gate and arguments match
        if last is not None and name in _FUSABLE and last.name == name and last.arg == arg:
            last.targets.extend(targets)
        else:
            self.ops.append(Op(name, targets, arg))
        return self

    def __add__(self, other: "StimCircuit") -> "StimCircuit":
        return StimCircuit(self.ops + other.ops)

    def __mul__(self, k: int) -> "StimCircuit":
        return StimCircuit([o for _ in range(int(k)) for o in self.ops])

    __rmul__ = __mul__

    def __len__(self):
        return len(self.ops)

    @property
    def num_qubits(self) -> int:
        q = [t for o in self.ops if o.name not in _ANNOT for t in o.targets]
        return (max(q) + 1) if q else 0

    @property
    def num_measurements(self) -> int:
        return sum(len(o.targets) for o in self.ops if o.name in ("M", "MR", "MX"))

    @property
    def num_detectors(self) -> int:
        return sum(1 for o in self.ops if o.name == "DETECTOR")

    @property
    def num_observables(self) -> int:
        ks = [int(o.arg) for o in self.ops if o.name == "OBSERVABLE_INCLUDE"]
        return (max(ks) + 1) if ks else 0

    def __str__(self):
        out = []
        for o in self.ops:
            a = "" if o.arg is None else f"({o.arg:g})"
            if o.name in ("DETECTOR", "OBSERVABLE_INCLUDE"):
                t = " ".join(f"rec[{k}]" for k in o.targets)
            else:
                t = " ".join(str(k) for k in o.targets)
            out.append(f"{o.name}{a} {t}".rstrip())
        return "\n".join(out) + "\n"

    def detector_error_model(self, flatten_loops: bool = True) -> "DetectorErrorModel":
        return detector_error_model(self)


def add_cx_error(circuit: StimCircuit, p: float) -> StimCircuit:
    """``AddCXError(circuit, 'DEPOLARIZE2(%f)' % p)`` (``src/ErrorPlugin.py:11-25``): every CX
    instruction is followed by a DEPOLARIZE2 on the same target list.  The reference formats the
    probability with ``%f`` (6 decimals) before stim parses it back: kept."""
    pf = float("%f" % p)
    ops = []
    for o in circuit.ops:
        ops.append(Op(o.name, list(o.targets), o.arg))
        if o.name == "CX":
            ops.append(Op("DEPOLARIZE2", list(o.targets), pf))
    return StimCircuit(ops)


# ------------------------------------------------------------------------------------ the DEM
def depolarize1_component(p: float) -> float:
    """Independent per-Pauli probability of ``DEPOLARIZE1(p)`` (X, Y, Z each; exact)."""
    if p > 0.75:
        raise ValueError("DEPOLARIZE1 probability above 3/4")
    return 0.5 - 0.5 * math.sqrt(1.0 - (4.0 * p) / 3.0)


def depolarize2_component(p: float) -> float:
    """Independent per-Pauli probability of ``DEPOLARIZE2(p)`` (15 non-identity Paulis; exact)."""
    if p > 15.0 / 16.0:
        raise ValueError("DEPOLARIZE2 probability above 15/16")
    return 0.5 - 0.5 * (1.0 - (16.0 * p) / 15.0) ** 0.125


@dataclass
class DetectorErrorModel:
    """``probs[j]``, ``dets[j]`` (sorted detector indices) and ``obs[j]`` (observable indices) of each
    independent error mechanism; ``det_segment[d]`` = the number of ``SHIFT_COORDS`` before detector
    d was declared (stim's ``shift_detectors`` lines)."""

    num_detectors: int
    num_observables: int
    num_shifts: int = 0
    probs: list = field(default_factory=list)
    dets: list = field(default_factory=list)
    obs: list = field(default_factory=list)
    det_segment: list = field(default_factory=list)

    @property
    def num_errors(self) -> int:
        return len(self.probs)

    def check_matrix(self) -> np.ndarray:
        """Dense [num_detectors x num_errors] uint8."""
        H = np.zeros((self.num_detectors, self.num_errors), np.uint8)
        for j, ds in enumerate(self.dets):
            H[list(ds), j] = 1
        return H

    def observable_matrix(self) -> np.ndarray:
        L = np.zeros((self.num_observables, self.num_errors), np.uint8)
        for j, ks in enumerate(self.obs):
            L[list(ks), j] = 1
        return L

    def __str__(self):
        """stim-style text (errors first, then the detector / shift lines in circuit order), with
        exact ``repr`` probabilities."""
        return self.to_text("exact")

    def stim_order(self) -> list:
        """Mechanism indices in the order stim lists one flush of its error classes: ascending by the
        target list, detectors before observables, a prefix before its extensions (``error(0.125) D0``,
        ``error(0.375) D0 D1``, ``error(0.25) D1`` in stim's ``detector_error_model`` docstring)."""
        return sorted(range(self.num_errors), key=lambda j: (list(self.dets[j]) + [1 << 40 | k for k in self.obs[j]]))

    def to_text(self, style: str = "exact") -> str:
        """The DEM as the text ``GenFaultHyperGraph`` parses (``str(dem)``, ``src/Simulators_SpaceTime.py:950``):
        every ``error(p) D.. L..`` line first, then the ``shift_detectors(1) 0`` / ``detector`` lines in
        circuit order.

        ``style="exact"``: this model's mechanism order, probabilities as ``repr`` (round-trip exact).
        ``style="stim"``: stim's text as the reference saw it — mechanisms in :meth:`stim_order`, each
        probability through C++'s default stream format (6 significant digits, ``%g``: exponent
        notation below 1e-4), detector lines with their coordinate ``detector(0) Dk``.  Against stim
        itself this rendering is parity unpinned (stim is absent); it is what ``compat=True`` parses."""
        if style not in ("exact", "stim"):
            raise ValueError(f"unknown DEM text style {style!r}")
        order = self.stim_order() if style == "stim" else range(self.num_errors)
        fmt = (lambda p: format(p, "g")) if style == "stim" else repr
        lines = [f"error({fmt(self.probs[j])}) " + " ".join([f"D{d}" for d in self.dets[j]] + [f"L{k}" for k in self.obs[j]])
                 for j in order]
        det = "detector(0) D{}" if style == "stim" else "detector D{}"
        seg = 0
        for d, s in enumerate(self.det_segment):
            while seg < s:
                lines.append("shift_detectors(1) 0")
                seg += 1
            lines.append(det.format(d))
        lines += ["shift_detectors(1) 0"] * (self.num_shifts - seg)
        return "\n".join(lines)

    @classmethod
    def from_text(cls, text: str, compat: bool = False) -> "DetectorErrorModel":
        """Parse DEM text the way ``GenFaultHyperGraph`` reads it (``src/Simulators_SpaceTime.py:554-583``):
        error lines in order, detectors from the ``detector`` lines, segments from the
        ``shift_detectors(1) 0`` lines.  ``compat=True`` reads each probability with the reference's
        ``float(re.findall("\\d+\\.\\d+", token)[0])`` (``:575, :642``): a probability printed in
        exponent notation keeps only its mantissa (``6.67e-05`` -> 6.67) and one printed without a
        decimal point raises ``IndexError``, as the reference does; ``compat=False`` reads the number
        exactly."""
        import re

        items = text.split("\n")
        dem = cls(0, 0)
        D = K = seg = 0
        for it in items:
            tok = it.split()
            if not tok:
                continue
            if "error" in it:
                head = tok[0]
                if compat:
                    p = float(re.findall(r"\d+\.\d+", head)[0])
                else:
                    p = float(head[head.index("(") + 1:head.rindex(")")])
                ds = sorted(int(t[1:]) for t in tok[1:] if t.startswith("D"))
                ks = sorted(int(t[1:]) for t in tok[1:] if t.startswith("L"))
                dem.probs.append(p)
                dem.dets.append(tuple(ds))
                dem.obs.append(tuple(ks))
                K = max([K] + [k + 1 for k in ks])
                D = max([D] + [d + 1 for d in ds])
            elif it.strip() == "shift_detectors(1) 0":
                seg += 1
            elif "detector" in it and "shift" not in it:
                d = int(tok[1][1:])
                while len(dem.det_segment) <= d:
                    dem.det_segment.append(seg)
                D = max(D, d + 1)
        dem.num_detectors, dem.num_observables, dem.num_shifts = D, K, seg
        return dem


_PAULI2 = [(a, b) for a in range(4) for b in range(4) if (a, b) != (0, 0)]  # 0 I, 1 X, 2 Y, 3 Z


def detector_error_model(circuit: StimCircuit) -> DetectorErrorModel:
    """Backward Pauli-frame analysis of a flattened circuit (see the module docstring)."""
    ops = circuit.ops
    # forward pass: measurement records, detectors, observables
    nrec = 0
    rec_of = []  # per op: first record index (measurements)
    det_recs, obs_recs, det_seg = [], {}, []
    seg = 0
    for o in ops:
        rec_of.append(nrec)
        if o.name in ("M", "MR", "MX"):
            nrec += len(o.targets)
        elif o.name == "DETECTOR":
            det_recs.append([nrec + k for k in o.targets])
            det_seg.append(seg)
        elif o.name == "OBSERVABLE_INCLUDE":
            obs_recs.setdefault(int(o.arg), []).extend(nrec + k for k in o.targets)
        elif o.name == "SHIFT_COORDS":
            seg += 1
    D = len(det_recs)
    K = (max(obs_recs) + 1) if obs_recs else 0
    sens = [0] * nrec  # record -> bitset of detectors (bits 0..D-1) and observables (D..D+K-1)
    for d, rs in enumerate(det_recs):
        for r in rs:
            if r < 0:
                raise ValueError("detector refers to a measurement before the circuit start")
            sens[r] ^= 1 << d
    for k, rs in obs_recs.items():
        for r in rs:
            sens[r] ^= 1 << (D + k)
    nq = max(circuit.num_qubits, 1)
    SX, SZ = [0] * nq, [0] * nq
    found = {}  # symptom bitset -> [probability, earliest op index]

    def add(sym: int, p: float, t: int):
        if sym == 0 or p <= 0.0:
            return
        cur = found.get(sym)
        if cur is None:
            found[sym] = [p, t]
        else:
            cur[0] = cur[0] * (1.0 - p) + p * (1.0 - cur[0])
            cur[1] = t

    for t in range(len(ops) - 1, -1, -1):
        o = ops[t]
        nm, tg = o.name, o.targets
        if nm in _ANNOT:
            continue
        if nm in ("M", "MR", "MX"):
            base = rec_of[t]
            for i in range(len(tg) - 1, -1, -1):
                q, s = tg[i], sens[base + i]
                if nm == "MR":
                    SX[q], SZ[q] = s, 0
                elif nm == "M":
                    SX[q] ^= s
                else:
                    SZ[q] ^= s
        elif nm in ("R", "RX"):
            for q in tg:
                SX[q] = SZ[q] = 0
        elif nm == "H":
            for q in tg:
                SX[q], SZ[q] = SZ[q], SX[q]
        elif nm == "CX":
            if len(tg) % 2:
                raise ValueError("CX needs target pairs")
            for i in range(len(tg) - 2, -1, -2):
                c, x = tg[i], tg[i + 1]
                SX[c] ^= SX[x]
                SZ[x] ^= SZ[c]
        elif nm == "DEPOLARIZE1":
            pc = depolarize1_component(o.arg)
            for q in tg:
                add(SX[q], pc, t)
                add(SX[q] ^ SZ[q], pc, t)
                add(SZ[q], pc, t)
        elif nm == "DEPOLARIZE2":
            pc = depolarize2_component(o.arg)
            if len(tg) % 2:
                raise ValueError("DEPOLARIZE2 needs target pairs")
            for i in range(0, len(tg), 2):
                a, b = tg[i], tg[i + 1]
                fa = (0, SX[a], SX[a] ^ SZ[a], SZ[a])
                fb = (0, SX[b], SX[b] ^ SZ[b], SZ[b])
                for pa, pb in _PAULI2:
                    add(fa[pa] ^ fb[pb], pc, t)
        elif nm == "X_ERROR":
            for q in tg:
                add(SX[q], o.arg, t)
        elif nm == "Z_ERROR":
            for q in tg:
                add(SZ[q], o.arg, t)
    dem = DetectorErrorModel(D, K, num_shifts=seg, det_segment=det_seg)
    mask_d = (1 << D) - 1
    for sym, (p, _) in sorted(found.items(), key=lambda kv: (kv[1][1], _bits(kv[0]))):
        dem.probs.append(p)
        dem.dets.append(tuple(_bits(sym & mask_d)))
        dem.obs.append(tuple(b - D for b in _bits(sym >> D << D)))
    return dem


def _bits(x: int) -> list:
    out = []
    while x:
        low = x & -x
        out.append(low.bit_length() - 1)
        x ^= low
    return out


# ------------------------------------------------------------------- the fault hypergraphs
def _layers(dem: DetectorErrorModel):
    """The reference's first and last detector layers (``src/Simulators_SpaceTime.py:557-572``):
    per-cycle counts from the ``shift_detectors`` positions; layer 0 = the first cycle's
    detectors, layer 1 = the last ``len(detectors) - Σ`` (earlier cycles)."""
    D = dem.num_detectors
    counts = [sum(1 for s in dem.det_segment if s == k) for k in range(1, dem.num_shifts)]
    counts.append(D - int(np.sum(counts)))
    first = list(range(counts[0]))
    last = list(range(D - counts[-1], D))
    return first, last


def _error_layers(dem: DetectorErrorModel, layers):
    sets = [set(L) for L in layers]
    out = []
    for j in range(dem.num_errors):
        ds = set(dem.dets[j])
        occ = [i for i, s in enumerate(sets) if ds & s]
        out.append(occ[0] if occ else None)
    return out


def GenFaultHyperGraph(detector_error_model: DetectorErrorModel, num_rounds: int, num_rep: int, num_logicals: int):
    """``src/Simulators_SpaceTime.py:551-610``: (H_list, L_list, channel_prob_list) of the first and
    last detector layers.  An error belongs to the first layer it touches, restricted to that
    layer's detectors; errors touching neither are dropped."""
    dem = _as_dem(detector_error_model)
    layers = _layers(dem)
    lay = _error_layers(dem, layers)
    H_list, L_list, P_list = [], [], []
    for li, dl in enumerate(layers):
        cols = [j for j in range(dem.num_errors) if lay[j] == li]
        pos = {d: i for i, d in enumerate(dl)}
        H = np.zeros((len(dl), len(cols)))
        L = np.zeros((num_logicals, len(cols)))
        for c, j in enumerate(cols):
            for d in dem.dets[j]:
                if d in pos:
                    H[pos[d], c] = 1
            for k in dem.obs[j]:
                if k < num_logicals:
                    L[k, c] = 1
        H_list.append(H)
        L_list.append(L)
        P_list.append([dem.probs[j] for j in cols])
    return H_list, L_list, P_list


def GenCorrecHyperGraph(detector_error_model: DetectorErrorModel, num_rounds: int, num_rep: int, num_checks: int,
                        num_logicals: int):
    """``src/Simulators_SpaceTime.py:615-668``: the space correction matrix of the first layer's
    errors, ``Σ_{i=0..num_rep} H[i·m:(i+1)·m] mod 2`` over the first and last layers' detectors."""
    dem = _as_dem(detector_error_model)
    layers = _layers(dem)
    lay = _error_layers(dem, layers)
    relevant = layers[0] + layers[1]
    pos = {d: i for i, d in enumerate(relevant)}
    cols = [j for j in range(dem.num_errors) if lay[j] == 0]
    H = np.zeros((len(relevant), len(cols)))
    for c, j in enumerate(cols):
        for d in dem.dets[j]:
            if d in pos:
                H[pos[d], c] = 1
    Hs = np.zeros((num_checks, len(cols)))
    for i in range(num_rep + 1):
        Hs += H[i * num_checks:(i + 1) * num_checks, :]
    return Hs % 2


def _as_dem(x, compat: bool = True) -> DetectorErrorModel:
    """A DEM object as is; DEM text (``str(...)`` of one, or stim's format) parsed the reference's way
    (:meth:`DetectorErrorModel.from_text`, the reference's probability regex unless ``compat=False``)."""
    if isinstance(x, DetectorErrorModel):
        return x
    if isinstance(x, str):
        return DetectorErrorModel.from_text(x, compat=compat)
    raise TypeError("expected a DetectorErrorModel or its text (stim is absent; build it with detector_error_model())")


def misparsed_mechanisms(dem: DetectorErrorModel) -> list:
    """Indices of the mechanisms whose probability the reference's ``\\d+\\.\\d+`` parse of stim's text
    (6 significant digits, exponent notation below 1e-4) does not read back within that rounding:
    the ones printed in exponent notation, which it reads as their mantissa (``5.33e-05`` -> 5.33)."""
    out = []
    for j, p in enumerate(dem.probs):
        s = format(p, "g")
        if "e" in s or "." not in s:
            out.append(j)
    return out


# ------------------------------------------------------------------- CX schedules
def _bipartite_graph(H):
    """``BipartitieGraphFromCheckMat`` (``src/CircuitScheduling.py:11-22``): check i is node -(i+1),
    bit j is node j+1; edges in row-major order."""
    import networkx as nx

    H = np.asarray(H)
    m, n = H.shape
    G = nx.Graph()
    G.add_nodes_from(list(-np.arange(1, m + 1)), bipartite=0)
    G.add_nodes_from(list(np.arange(1, n + 1)), bipartite=1)
    G.add_edges_from([(-(i + 1), j + 1) for i in range(m) for j in range(n) if H[i][j] == 1])
    return G


def _regularize(G):
    """``TransformBipartiteGraph`` (``:31-70``): dummy check nodes up to the bit count, then dummy
    edges (first open check, first open bit without that edge, in dict order) until every node has
    the maximum degree."""
    Gs = copy.deepcopy(G)
    C = list({v for v, d in G.nodes(data=True) if d["bipartite"] == 0})
    V = list(set(G) - set(C))
    Gs.add_nodes_from(list(-np.arange(len(C) + 1, len(V) + 1)), bipartite=0)
    delta = max(dict(Gs.degree).values())
    open_deg = {v: d for v, d in dict(Gs.degree()).items() if d < delta}
    while open_deg:
        progressed = False
        for c in list(open_deg.keys()):
            if c >= 0 or c not in open_deg:
                continue
            for v in list(open_deg.keys()):
                if v > 0 and not Gs.has_edge(c, v):
                    Gs.add_edge(c, v)
                    progressed = True
                    for u in (c, v):
                        if open_deg[u] + 1 == delta:
                            open_deg.pop(u)
                        else:
                            open_deg[u] += 1
                    break
        if not progressed:
            raise RuntimeError("bipartite regularization made no progress")
    return Gs


def ColorationCircuit(H):
    """``src/CircuitScheduling.py:102-110``: edge colouring by repeated maximum matchings of the
    regularized Tanner graph; time step t maps check -> data qubit."""
    from networkx.algorithms import bipartite

    G = _bipartite_graph(H)
    Gs = _regularize(G)
    C = list({v for v, d in G.nodes(data=True) if d["bipartite"] == 0})
    Cs = list({v for v, d in Gs.nodes(data=True) if d["bipartite"] == 0})
    out = []
    while len(Gs.edges()) > 0:
        top = list({v for v, d in Gs.nodes(data=True) if d["bipartite"] == 0})
        bm = bipartite.matching.hopcroft_karp_matching(Gs, top)
        out.append({-int(c) - 1: int(bm[c]) - 1 for c in bm if c in C})
        Gs.remove_edges_from([(c, bm[c]) for c in bm if c in Cs])
    return out


def RandomCircuit(H):
    """``src/CircuitScheduling.py:116-131``: per check a shuffled support (``random.Random(i +
    30000)``), time step t takes each check's t-th data qubit."""
    H = np.asarray(H)
    m, n = H.shape
    wmax = max(int(np.sum(H[i, :])) for i in range(m))
    sup = [list(np.where(H[i, :] == 1)[0]) for i in range(m)]
    for i in range(m):
        random.Random(i + 30000).shuffle(sup[i])
    out = []
    for t in range(wmax):
        out.append({i: int(sup[i][t]) for i in range(m) if len(sup[i]) >= t + 1})
    return out


# ------------------------------------------------------------------- the reference's circuits
def syndrome_circuits(hx, hz, lx, error_params: dict, pz: float, num_rounds: int, num_rep: int, scheduling_X,
                      scheduling_Z):
    """``CodeSimulator_Circuit_SpaceTime._generate_circuit`` (``src/Simulators_SpaceTime.py:737-940``):
    (noisy full circuit, noisy fault circuit).  Qubits: data 0..n-1, Z ancillas n..n+m_z-1, X
    ancillas after them.  X-stabilizer measurements are the detectors (raw in a round's first
    repetition, differenced with the previous repetition after it); the final MX of the data gives
    the last syndrome (raw in the full circuit, differenced in the fault circuit) and the
    observables ``lx``."""
    hx, hz, lx = (np.asarray(a) for a in (hx, hz, lx))
    n = hx.shape[1]
    data = list(range(n))
    nZ, nX = hz.shape[0], hx.shape[0]
    Za = list(range(n, n + nZ))
    Xa = list(range(n + nZ, n + nZ + nX))
    ep = error_params

    init = StimCircuit()
    init.append("RX", data)
    init.append("R", Xa + Za)
    init.append("DEPOLARIZE1", data, pz)

    def rep_block(first: bool, tail_to: StimCircuit | None):
        c = StimCircuit()
        c.append("H", Xa)
        c.append("DEPOLARIZE1", Xa, ep["p_state_p"])
        c.append("DEPOLARIZE1", data, ep["p_i"])
        c.append("TICK")
        for step in scheduling_X:
            c.append("DEPOLARIZE1", data + Xa, ep["p_idling_gate"])
            for j in step:
                c.append("CX", [Xa[j], step[j]])
            c.append("TICK")
        c.append("DEPOLARIZE1", Za, ep["p_state_p"])
        c.append("DEPOLARIZE1", data, ep["p_i"])
        c.append("TICK")
        for step in scheduling_Z:
            c.append("DEPOLARIZE1", data + Za, ep["p_idling_gate"])
            for j in step:
                c.append("CX", [step[j], Za[j]])
            c.append("TICK")
        c.append("H", Xa)
        c.append("DEPOLARIZE1", Xa, ep["p_m"])
        c.append("DEPOLARIZE1", data, ep["p_i"])
        c.append("MR", Za + Xa)
        if first:
            c.append("SHIFT_COORDS", [], 1)
            for i in range(nX):
                c.append("DETECTOR", [-nX + i], 0)
            c.append("TICK")
        else:
            for i in range(nX):
                c.append("DETECTOR", [-nX + i, -nX + i - nZ - nX], 0)
            tail_to.append("TICK")  # (the reference appends this TICK to the first block, :867)
        return c

    rep1 = rep_block(True, None)
    rep2 = rep_block(False, rep1)
    stab = rep1 + (num_rep - 1) * rep2

    def final(diff: bool):
        c = StimCircuit()
        c.append("DEPOLARIZE1", data, ep["p_m"])
        c.append("MX", data)
        c.append("SHIFT_COORDS", [], 1)
        for i in range(nX):
            sup = list(np.where(hx[i, :] == 1)[0])
            recs = [-n + d for d in sup]
            if diff:
                recs.append(-nX + i - n)
            c.append("DETECTOR", recs, 0)
        for i in range(len(lx)):
            c.append("OBSERVABLE_INCLUDE", [-n + d for d in np.where(lx[i, :] == 1)[0]], i)
        return c

    circuit = init + num_rounds * stab + final(False)
    fault = init + stab + final(True)
    return add_cx_error(circuit, ep["p_CX"]), add_cx_error(fault, ep["p_CX"])
