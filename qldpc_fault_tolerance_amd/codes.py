"""CSS code objects, loaders and constructions for the decoding hot path.

The reference passes codes around as duck-typed objects with ``.hx .hz .lx .lz
.N .K`` (``bposd.hgp.hgp`` unpickled by ``load_object``, ``src/Simulators.py:69-71``,
or ``bposd.css.css_code`` built in the notebooks from ``scipy.io.loadmat``
matrices).  :class:`CSSCode` is the same duck type, backed by
dense ``uint8`` matrices plus cached CSR views for the device graph builder.

Loaders (nothing here executes code from a data file):

* ``.pkl``  – :mod:`.safepickle` opcode reader (never ``pickle.load``);
* ``.mat``  – ``scipy.io.loadmat`` (MATLAB v5 numeric arrays);
* ``.npy``  – ``numpy.load(allow_pickle=False)`` (also the reference's
  ``tanner_code1_h*.txt``, which are ``.npy`` files);
* ``.npz``  – this package's bundled CSR copies under ``codes_lib/``.

:func:`hgp` restates the hypergraph-product formula the reference gets from
``bposd.hgp.hgp`` (checked bit-for-bit against ``codes_lib/hgp_34_n225.pkl``).
:func:`random_biregular_check_matrix` restates ``RandomaGraphs`` +
the girth-raising swaps of ``src/QuantumExanderCodesGene.py:181-251,286-330``;
it is how the missing ``hgp_34_n1600`` / ``hgp_34_n1225_q3`` stand-ins are built
(``tools/synth_hgp_codes.py``).
"""
from __future__ import annotations

import os
import random as _pyrandom
from dataclasses import dataclass, field

import numpy as np

from . import gf2
from .safepickle import load_pickled_code_arrays

CODES_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "codes_lib")


# --------------------------------------------------------------------------- CSR
@dataclass
class CSR:
    """Binary sparse matrix, rows sorted by column (``mod2sparse`` row order)."""

    m: int
    n: int
    row_ptr: np.ndarray  # int32 [m+1]
    col_idx: np.ndarray  # int32 [nnz]

    @staticmethod
    def from_dense(H) -> "CSR":
        A = np.asarray(H)
        A = (A.astype(np.int64) % 2).astype(bool)
        m, n = A.shape
        rows, cols = np.nonzero(A)  # row-major, columns ascending within a row
        row_ptr = np.zeros(m + 1, dtype=np.int32)
        np.add.at(row_ptr, rows + 1, 1)
        row_ptr = np.cumsum(row_ptr).astype(np.int32)
        return CSR(m, n, row_ptr, cols.astype(np.int32))

    @property
    def nnz(self) -> int:
        return int(self.row_ptr[-1])

    def to_dense(self) -> np.ndarray:
        D = np.zeros((self.m, self.n), dtype=np.uint8)
        rows = np.repeat(np.arange(self.m), np.diff(self.row_ptr))
        D[rows, self.col_idx] = 1
        return D

    def row_degrees(self) -> np.ndarray:
        return np.diff(self.row_ptr)

    def col_degrees(self) -> np.ndarray:
        return np.bincount(self.col_idx, minlength=self.n)

    def matvec(self, v) -> np.ndarray:
        """``H @ v % 2`` for a 0/1 vector (or ``[B, n]`` batch)."""
        v = np.asarray(v).astype(np.uint8) & 1
        if v.ndim == 1:
            return np.bitwise_xor.reduceat(v[self.col_idx], self.row_ptr[:-1]) * (np.diff(self.row_ptr) > 0)
        g = v[:, self.col_idx]
        out = np.bitwise_xor.reduceat(g, self.row_ptr[:-1], axis=1)
        out[:, np.diff(self.row_ptr) == 0] = 0
        return out


# --------------------------------------------------------------------- CSS code
@dataclass
class CSSCode:
    """Duck type of ``bposd.css.css_code`` / ``bposd.hgp.hgp`` (``hx hz lx lz N K``)."""

    hx: np.ndarray
    hz: np.ndarray
    lx: np.ndarray
    lz: np.ndarray
    name: str = "<Unnamed CSS code>"
    h1: np.ndarray | None = None
    h2: np.ndarray | None = None
    _csr: dict = field(default_factory=dict, repr=False)

    def __post_init__(self):
        for a in ("hx", "hz", "lx", "lz"):
            setattr(self, a, (np.asarray(getattr(self, a)).astype(np.int64) % 2).astype(np.uint8))
        if self.hx.shape[1] != self.hz.shape[1]:
            raise ValueError("hx and hz must have the same number of columns")

    @property
    def N(self) -> int:
        return int(self.hx.shape[1])

    @property
    def K(self) -> int:
        return int(self.lx.shape[0])

    def csr(self, which: str) -> CSR:
        if which not in self._csr:
            self._csr[which] = CSR.from_dense(getattr(self, which))
        return self._csr[which]

    def test(self) -> bool:
        """Commutation checks (``hx hz^T = 0``, ``hx lz^T = 0``, ``hz lx^T = 0``, ``lx lz^T`` full rank)."""
        ok = not gf2.matmul(self.hx, self.hz.T).any()
        ok &= not gf2.matmul(self.hx, self.lz.T).any()
        ok &= not gf2.matmul(self.hz, self.lx.T).any()
        ok &= gf2.rank(gf2.matmul(self.lx, self.lz.T)) == self.K
        return bool(ok)

    @staticmethod
    def from_checks(hx, hz, name: str = "<Unnamed CSS code>", lx=None, lz=None) -> "CSSCode":
        if lx is None or lz is None:
            lx, lz = gf2.compute_logicals(hx, hz)
        return CSSCode(hx=hx, hz=hz, lx=lx, lz=lz, name=name)


def hgp(h1, h2=None, name: str | None = None) -> CSSCode:
    """Hypergraph product ``hx=[h1⊗I_n2 | I_m1⊗h2ᵀ]``, ``hz=[I_n1⊗h2 | h1ᵀ⊗I_m2]``.

    Same block layout as ``bposd.hgp.hgp`` (``hx1,hx2,hz1,hz2`` attributes of the
    reference pickle).  Logicals from :func:`gf2.compute_logicals`.
    """
    h1 = (np.asarray(h1).astype(np.int64) % 2).astype(np.uint8)
    h2 = h1 if h2 is None else (np.asarray(h2).astype(np.int64) % 2).astype(np.uint8)
    m1, n1 = h1.shape
    m2, n2 = h2.shape
    hx = np.hstack([np.kron(h1, np.eye(n2, dtype=np.uint8)), np.kron(np.eye(m1, dtype=np.uint8), h2.T)])
    hz = np.hstack([np.kron(np.eye(n1, dtype=np.uint8), h2), np.kron(h1.T, np.eye(m2, dtype=np.uint8))])
    code = CSSCode.from_checks(hx, hz, name=name or f"hgp[[{hx.shape[1]}]]")
    code.h1, code.h2 = h1, h2
    return code


# ---------------------------------------------------------------------- loaders
def load_npz(path: str) -> CSSCode:
    z = np.load(path, allow_pickle=False)

    def dense(prefix):
        m, n = (int(x) for x in z[prefix + "_shape"])
        return CSR(m, n, z[prefix + "_row_ptr"].astype(np.int32), z[prefix + "_col_idx"].astype(np.int32)).to_dense()

    code = CSSCode(hx=dense("hx"), hz=dense("hz"), lx=dense("lx"), lz=dense("lz"),
                   name=str(z["name"]) if "name" in z else os.path.basename(path))
    if "h1_shape" in z:
        code.h1 = dense("h1")
        code.h2 = dense("h2") if "h2_shape" in z else code.h1
    return code


def save_npz(code: CSSCode, path: str) -> None:
    arrs = {"name": np.array(code.name)}
    mats = {"hx": code.hx, "hz": code.hz, "lx": code.lx, "lz": code.lz}
    if code.h1 is not None:
        mats["h1"] = code.h1
        if code.h2 is not None and not np.array_equal(code.h2, code.h1):
            mats["h2"] = code.h2
    for k, M in mats.items():
        c = CSR.from_dense(M)
        arrs[k + "_shape"] = np.array([c.m, c.n], dtype=np.int64)
        arrs[k + "_row_ptr"] = c.row_ptr
        arrs[k + "_col_idx"] = c.col_idx.astype(np.int16 if c.n < 32768 else np.int32)
    np.savez_compressed(path, **arrs)


def load_pkl(path: str) -> CSSCode:
    """Drop-in for ``load_object`` on the reference's code pickles (no unpickling)."""
    d = load_pickled_code_arrays(path)
    missing = [k for k in ("hx", "hz", "lx", "lz") if not isinstance(d.get(k), np.ndarray)]
    if missing:
        raise ValueError(f"{path}: pickled code lacks arrays {missing}")
    code = CSSCode(hx=d["hx"], hz=d["hz"], lx=d["lx"], lz=d["lz"], name=str(d.get("name", "")))
    if isinstance(d.get("h1"), np.ndarray):
        code.h1 = (d["h1"].astype(np.int64) % 2).astype(np.uint8)
        if isinstance(d.get("h2"), np.ndarray):
            code.h2 = (d["h2"].astype(np.int64) % 2).astype(np.uint8)
    if "N" in d and d["N"] is not None and int(d["N"]) != code.N:
        raise ValueError("pickled N disagrees with hx")
    return code


def load_matrix(path: str, key: str | None = None) -> np.ndarray:
    """One parity-check matrix from ``.mat``/``.npy``/``.txt``(npy) as uint8."""
    ext = os.path.splitext(path)[1].lower()
    if ext == ".mat":
        import scipy.io

        d = scipy.io.loadmat(path)
        keys = [k for k in d if not k.startswith("__")]
        if key is None:
            if len(keys) != 1:
                raise ValueError(f"{path}: pass key= one of {keys}")
            key = keys[0]
        A = np.asarray(d[key])
    else:
        A = np.load(path, allow_pickle=False)
    return (A.astype(np.int64) % 2).astype(np.uint8)


def load_code(path: str, hz_path: str | None = None, name: str | None = None) -> CSSCode:
    """Load a code from the reference's ``codes_lib`` formats or a bundled ``.npz``.

    ``.pkl``/``.npz`` hold whole codes.  For ``.mat``/``.npy`` pass the ``hx``
    file as ``path`` and the ``hz`` file as ``hz_path`` (or pass ``..._hx.mat``
    alone and the ``_hz`` sibling is used); logicals are computed as
    ``css_code`` does.
    """
    ext = os.path.splitext(path)[1].lower()
    if ext == ".pkl":
        return load_pkl(path)
    if ext == ".npz":
        return load_npz(path)
    if hz_path is None:
        base = os.path.basename(path)
        if "_hx" not in base:
            raise ValueError("pass hz_path for a single-matrix file")
        hz_path = os.path.join(os.path.dirname(path), base.replace("_hx", "_hz"))
    hx = load_matrix(path)
    hz = load_matrix(hz_path)
    return CSSCode.from_checks(hx, hz, name=name or os.path.basename(path).replace("_hx", ""))


def bundled_codes() -> list:
    return sorted(f[:-4] for f in os.listdir(CODES_LIB) if f.endswith(".npz"))


def get_code(name: str) -> CSSCode:
    """A bundled code by name (``hgp_34_n225``, ``hgp_34_n1600``, ``GenBicycleA1`` …)."""
    p = os.path.join(CODES_LIB, name + ".npz")
    if not os.path.exists(p):
        raise KeyError(f"unknown bundled code {name!r}; have {bundled_codes()}")
    return load_npz(p)


# ----------------------------------------------------- space-time check matrix
def space_time_csr(h, t0: int) -> CSR:
    """CSR of ``GetSpaceTimeCheckMat(h, t0)`` (``src/Decoders_SpaceTime.py:179-194``).

    ``t0·m × t0·(n+m)``; block (i,i) = ``[h | I_m]``, block (i,i-1) = ``[0 | I_m]``.
    Rows keep ascending column order (so the ``I_m`` of block (i,i-1) comes first).
    """
    hc = h if isinstance(h, CSR) else CSR.from_dense(h)
    m, n = hc.m, hc.n
    w = n + m
    rows = []
    for i in range(t0):
        for r in range(m):
            cols = []
            if i >= 1:
                cols.append((i - 1) * w + n + r)
            cols.extend(int(c) + i * w for c in hc.col_idx[hc.row_ptr[r]:hc.row_ptr[r + 1]])
            cols.append(i * w + n + r)
            rows.append(cols)
    row_ptr = np.zeros(t0 * m + 1, dtype=np.int32)
    row_ptr[1:] = np.cumsum([len(c) for c in rows])
    col_idx = np.array([c for r in rows for c in r], dtype=np.int32)
    return CSR(t0 * m, t0 * w, row_ptr, col_idx)


# ------------------------------------------------ random (Δc,Δv) Tanner graphs
def tanner_girth(H: np.ndarray) -> int:
    """Girth of the Tanner graph of ``H`` (BFS from every node; 0 if acyclic)."""
    H = np.asarray(H)
    m, n = H.shape
    adj = [[] for _ in range(m + n)]
    for c, v in zip(*np.nonzero(H)):
        adj[int(c)].append(m + int(v))
        adj[m + int(v)].append(int(c))
    best = 10**9
    for s in range(m + n):
        dist = {s: 0}
        parent = {s: -1}
        frontier = [s]
        while frontier:
            nxt = []
            for u in frontier:
                for w in adj[u]:
                    if w not in dist:
                        dist[w] = dist[u] + 1
                        parent[w] = u
                        nxt.append(w)
                    elif parent[u] != w:
                        best = min(best, dist[u] + dist[w] + 1)
            if best <= 2 * (dist[frontier[0]] + 1):
                break
            frontier = nxt
    return 0 if best == 10**9 else best


def _girth_and_short_cycles(H: np.ndarray):
    return tanner_girth(H)


def random_biregular_check_matrix(n0: int, delta_c: int, delta_v: int, seed: int,
                                  min_girth: int = 6, max_tries: int = 10000,
                                  require_full_rank: bool = True) -> np.ndarray:
    """``n0·Δv × n0·Δc`` check matrix with row weight Δc and column weight Δv.

    Restates ``RandomaGraphs`` (configuration model over shuffled check/variable
    ports, ``src/QuantumExanderCodesGene.py:181-233``), rejects multi-edges, then
    applies random double-edge swaps that never lower the girth, as
    ``RandSwapEdges1`` (``:286-310``) does, until ``min_girth`` is reached.
    ``require_full_rank`` keeps instances whose HGP has the reference's K
    (``[[1600,64]]``, ``[[1225,49]]``: ``Threshold-checkpoint.ipynb:233-236``).
    """
    rng = _pyrandom.Random(seed)
    m, n = n0 * delta_v, n0 * delta_c
    for _ in range(max_tries):
        cports = [c for c in range(m) for _ in range(delta_c)]
        vports = [v for v in range(n) for _ in range(delta_v)]
        rng.shuffle(cports)
        rng.shuffle(vports)
        H = np.zeros((m, n), dtype=np.int64)
        for c, v in zip(cports, vports):
            H[c, v] += 1
        # remove multi-edges by swaps with random single edges
        for _sw in range(10 * m * delta_c):
            multi = np.argwhere(H > 1)
            if multi.size == 0:
                break
            c1, v1 = multi[rng.randrange(len(multi))]
            ones = np.argwhere(H == 1)
            c2, v2 = ones[rng.randrange(len(ones))]
            if c2 == c1 or v2 == v1 or H[c1, v2] or H[c2, v1]:
                continue
            H[c1, v1] -= 1
            H[c2, v2] -= 1
            H[c1, v2] += 1
            H[c2, v1] += 1
        if (H > 1).any():
            continue
        g = _girth_and_short_cycles(H)
        for _sw in range(20000):
            if g >= min_girth:
                break
            edges = np.argwhere(H == 1)
            (c1, v1), (c2, v2) = edges[rng.randrange(len(edges))], edges[rng.randrange(len(edges))]
            if c1 == c2 or v1 == v2 or H[c1, v2] or H[c2, v1]:
                continue
            H2 = H.copy()
            H2[c1, v1] = H2[c2, v2] = 0
            H2[c1, v2] = H2[c2, v1] = 1
            g2 = _girth_and_short_cycles(H2)
            if g2 >= g:
                H, g = H2, g2
        if g < min_girth:
            continue
        Hu = H.astype(np.uint8)
        if require_full_rank and gf2.rank(Hu) != m:
            continue
        return Hu
    raise RuntimeError("could not build a biregular check matrix with the requested properties")
