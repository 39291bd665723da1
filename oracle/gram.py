"""Builder-defined factor-correlation GEMM + greedy pruning.

Test infrastructure only (see oracle/__init__.py).  PARITY UNPINNED: the reference
has no pruning code (only the docstring at factor_selector.py:30 and unused
``scipy.cluster.hierarchy`` imports, pipeline.ipynb:38-39).  The nearest reference
arithmetic is ``np.cov`` over factor returns (factor_selection_methods.py:73).

Spec (our own):
* ``Z[f,d,a]`` = per-date cross-sectional z-score of factor f (mean / std ddof=0 over
  non-NaN assets, as cs_zscore operations.py:77-78), NaN -> 0, rows with sigma in
  {0, NaN} -> 0.  ``M[f,d,a]`` = 1 where the exposure is non-NaN (and sigma > 0).
* ``C = (sum_d Z_d^T Z_d) / (sum_d M_d^T M_d)`` (0 where no pair is valid).
* Greedy pruning: walk factors in the given order (rank_IC_IR descending); keep f iff
  ``max_{k kept} |C[f,k]| < rho``; stop after ``top_x`` kept (if given).
"""
from __future__ import annotations

import numpy as np

from . import numerics as nm


def zscore_exposures(X):
    """X[F][D][A] -> (Z, M) as float64 arrays of the same shape."""
    v = np.asarray(X, dtype=np.float64)
    mu = nm.nanmean(v)
    sd = nm.nanstd(v, 0)
    with np.errstate(all="ignore"):
        z = (v - mu[..., None]) / sd[..., None]
    ok = (sd > 0) & ~np.isnan(sd)
    m = ~np.isnan(v) & ok[..., None]
    return np.where(m, z, 0.0), m.astype(np.float64)


def corr_matrix(X, d0=0, d1=None):
    Z, M = zscore_exposures(X)
    F, D, A = Z.shape
    d1 = D if d1 is None else d1
    Zf = Z[:, d0:d1].reshape(F, -1)
    Mf = M[:, d0:d1].reshape(F, -1)
    G = Zf @ Zf.T
    N = Mf @ Mf.T
    with np.errstate(all="ignore"):
        C = np.where(N > 0, G / N, 0.0)
    return C


EX_LIMBS, EX_FRAC = 6, 64      # csrc/exactsum.hpp: 6 x 32-bit payload limbs, LSB 2^-64
EX_SLOTS = EX_LIMBS + 1        # + invalid-term flag


def ex_fold(parts):
    """Restatement of csrc/exactsum.hpp ex_add over axis 0: float64 [U, ...] -> int64
    [EX_SLOTS, ...], each term truncated toward zero at 2^-64 and split into 32-bit
    chunks (exact integer sums, so any grouping of the U terms gives the same limbs)."""
    x = np.ascontiguousarray(parts, dtype=np.float64)
    u = x.view(np.uint64)
    neg = (u >> np.uint64(63)) != 0
    ex = ((u >> np.uint64(52)) & np.uint64(0x7FF)).astype(np.int64)
    man = u & np.uint64((1 << 52) - 1)
    bad = ex == 0x7FF
    M = np.where(ex == 0, man, man | np.uint64(1 << 52))
    E = np.where(ex == 0, -1074, ex - 1075)
    s = E + EX_FRAC
    bad |= (s + 53 > 32 * EX_LIMBS - 1) & (M != 0)
    M = np.where(bad, np.uint64(0), M)
    out = np.zeros((EX_SLOTS,) + x.shape[1:], dtype=np.int64)
    mask = np.uint64(0xFFFFFFFF)
    for k in range(EX_LIMBS):
        t = s - 32 * k
        left = (t >= 0) & (t < 32)
        right = (t < 0) & (t > -64)
        cl = (M << np.clip(t, 0, 31).astype(np.uint64)) & mask
        cr = (M >> np.clip(-t, 0, 63).astype(np.uint64)) & mask
        c = np.where(left, cl, np.where(right, cr, np.uint64(0))).astype(np.int64)
        out[k] = np.where(neg, -c, c).sum(axis=0)
    out[EX_LIMBS] = bad.sum(axis=0)
    return out


def ex_value(limbs):
    """csrc/exactsum.hpp ex_value: carry-normalise, then Horner from the top limb."""
    a = np.array(limbs, dtype=np.int64)
    carry = np.zeros(a.shape[1:], dtype=np.int64)
    for k in range(EX_LIMBS - 1):
        v = a[k] + carry
        lo = v & np.int64(0xFFFFFFFF)
        carry = (v - lo) >> np.int64(32)
        a[k] = lo
    a[EX_LIMBS - 1] += carry
    r = a[EX_LIMBS - 1].astype(np.float64)
    for k in range(EX_LIMBS - 2, -1, -1):
        r = r * 4294967296.0 + a[k].astype(np.float64)
    r = r * 2.0 ** -EX_FRAC
    return np.where(a[EX_LIMBS] != 0, np.nan, r)


def gram_exact_parts(Z, M, d0=0, d1=None):
    """Exact-fold form of the Gram over dates [d0, d1): (limbs [EX_SLOTS][F][F], counts
    [F][F] int64).  The unit of the fold is one date (Z_d^T Z_d by BLAS), so the result does
    not depend on how the dates are split over ranks."""
    F, D, A = Z.shape
    d1 = D if d1 is None else d1
    if d1 <= d0:
        return np.zeros((EX_SLOTS, F, F), np.int64), np.zeros((F, F), np.int64)
    Zt = np.ascontiguousarray(Z[:, d0:d1].transpose(1, 0, 2))          # [D'][F][A]
    parts = np.matmul(Zt, Zt.transpose(0, 2, 1))                       # per-date Z_d Z_d^T
    Mt = np.ascontiguousarray(M[:, d0:d1].transpose(1, 0, 2)).astype(np.int64)
    counts = np.einsum("dfa,dga->fg", Mt, Mt)
    return ex_fold(parts), counts


def gram_exact_finalize(limbs, counts):
    G = ex_value(limbs)
    G = np.triu(G) + np.triu(G, 1).T
    return G, counts.astype(np.float64)


def greedy_prune(C, order, rho=0.7, top_x=None):
    kept = []
    for f in order:
        if kept and np.max(np.abs(C[f, kept])) >= rho:
            continue
        kept.append(int(f))
        if top_x is not None and len(kept) >= top_x:
            break
    return kept
