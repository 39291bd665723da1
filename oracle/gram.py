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


def greedy_prune(C, order, rho=0.7, top_x=None):
    kept = []
    for f in order:
        if kept and np.max(np.abs(C[f, kept])) >= rho:
            continue
        kept.append(int(f))
        if top_x is not None and len(kept) >= top_x:
            break
    return kept
