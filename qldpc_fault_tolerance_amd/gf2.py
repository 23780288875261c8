"""GF(2) linear algebra on dense 0/1 matrices (host side, numpy).

Used at code-load time only (never on the shot path): ranks for code parameters
``K = N - rank(hx) - rank(hz)``, kernels/row bases for the logical operators of
codes that ship only ``hx``/``hz`` (the ``.mat`` LP/GBC files), and checks on the
synthesised HGP stand-ins.

The logical-operator construction restates the algorithm the reference relies on
through ``bposd.css.css_code`` (called by the notebooks after ``scipy.io.loadmat``,
SURVEY.md §3.4): ``lz`` = the vectors of a kernel basis of ``hx`` that are pivots
when appended below a row basis of ``hz``.  Any complement basis gives identical
failure flags in the simulators (``any(lz @ r % 2)`` for ``r`` in ker(hz) is
basis-independent), see DESIGN.md §"Logical operators".
"""
from __future__ import annotations

import numpy as np


def _as_u8(M) -> np.ndarray:
    A = np.asarray(M)
    if A.ndim != 2:
        raise ValueError("GF(2) matrix must be 2-D")
    return (A.astype(np.int64) % 2).astype(np.uint8)


def row_echelon(M, full: bool = False):
    """Row-reduce ``M`` over GF(2).

    Returns ``(R, rank, pivot_cols)`` with ``R`` in row-echelon form (reduced if
    ``full``).  Pivot search runs column by column, choosing the first row at or
    below the current rank with a 1 (the textbook order used by ``ldpc.mod2``).
    """
    R = _as_u8(M).copy()
    m, n = R.shape
    rank = 0
    pivots = []
    for c in range(n):
        if rank == m:
            break
        col = R[rank:, c]
        nz = np.flatnonzero(col)
        if nz.size == 0:
            continue
        p = rank + int(nz[0])
        if p != rank:
            R[[rank, p]] = R[[p, rank]]
        if full:
            rows = np.flatnonzero(R[:, c])
            rows = rows[rows != rank]
        else:
            rows = rank + 1 + np.flatnonzero(R[rank + 1:, c])
        if rows.size:
            R[rows] ^= R[rank]
        pivots.append(c)
        rank += 1
    return R, rank, pivots


def rank(M) -> int:
    return row_echelon(M)[1]


def row_basis(M) -> np.ndarray:
    """Rows of ``M`` that form a basis of its row space (echelon rows)."""
    R, r, _ = row_echelon(M)
    return R[:r]


def nullspace(M) -> np.ndarray:
    """Basis (as rows) of ker(M) = {v : M v = 0 mod 2}."""
    A = _as_u8(M)
    m, n = A.shape
    R, r, piv = row_echelon(A, full=True)
    pivset = set(piv)
    free = np.array([c for c in range(n) if c not in pivset], dtype=np.int64)
    basis = np.zeros((free.size, n), dtype=np.uint8)
    if free.size:
        basis[np.arange(free.size), free] = 1
        if r:
            # x_pivot(row) = sum over free f of R[row, f] x_f
            basis[:, np.asarray(piv, dtype=np.int64)] = R[:r][:, free].T
    return basis


def compute_lz(hx, hz) -> np.ndarray:
    """Z-type logicals: in ker(hx) and not in rowspace(hz).

    Restates ``bposd.css.css_code.compute_logicals.compute_lz`` (third-party,
    not vendored; used by the reference notebooks through ``css_code``).
    """
    ker_hx = nullspace(hx)
    im_hzT = row_basis(hz)
    stack = np.vstack([im_hzT, ker_hx])
    _, _, piv = row_echelon(stack.T)
    pivset = set(piv)
    idx = [i for i in range(im_hzT.shape[0], stack.shape[0]) if i in pivset]
    return stack[idx].astype(np.uint8)


def compute_logicals(hx, hz):
    """Return ``(lx, lz)`` for the CSS code (hx, hz)."""
    lx = compute_lz(hz, hx)
    lz = compute_lz(hx, hz)
    return lx, lz


def matmul(A, B) -> np.ndarray:
    return (np.asarray(A, dtype=np.int64) @ np.asarray(B, dtype=np.int64) % 2).astype(np.uint8)
