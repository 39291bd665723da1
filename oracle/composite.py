"""Oracle restatement of composite_factor.py (composite_factor_calculation,
weighted_composite_factor).  Test infrastructure only (see oracle/__init__.py).

``X[F][D][A]`` dense panel (all (date, symbol) rows present), factor ``names``.
"""
from __future__ import annotations

import numpy as np

from . import numerics as nm

SUFFIX = {  # composite_factor.py:158-163 / :244-249
    "_eq": (10, 90), "_flx": (2, 98), "_long": (2, 98), "_short": (2, 98),
}


def _scale(suffix, s, lo, hi):
    with np.errstate(all="ignore"):
        if suffix == "_eq":
            return np.where(s <= lo, -1.0, np.where(s >= hi, 1.0, 0.0))
        c = np.clip(s, lo, hi)
        if suffix == "_flx":
            return ((c - lo) / (hi - lo)) * 2 - 1
        if suffix == "_long":
            return (c - lo) / (hi - lo)
        return (c - hi) / (hi - lo)


def _pct(clean, p):
    s = np.sort(clean)
    q = np.true_divide(np.asarray([p], dtype=np.float64), 100)[0]
    return nm.percentile_linear(s, q)


def _prefix_groups(names):
    groups = {}
    for k, n in enumerate(names):
        groups.setdefault(n.split("_", 1)[0], []).append(k)
    return groups


def _rowmean_skipna(M):
    """DataFrame.mean(axis=1) skipna over columns ``M[k][A]`` -> [A]."""
    return nm.nanmean(np.ascontiguousarray(M.T))


def _safe_z(v):
    mu = nm.nanmean(v[None, :])[0]
    sd = nm.nanstd(v[None, :], 0)[0]
    if sd == 0 or np.isnan(sd):
        return np.zeros_like(v)
    return (v - mu) / sd


def _rank01(v):
    """(scipy.stats.rankdata(x) - 1) / (len - 1); any NaN -> all NaN (scipy>=1.10)."""
    n = len(v)
    if np.isnan(v).any():
        return np.full(n, np.nan)
    with np.errstate(all="ignore"):
        return (nm.rank_1d(v, "average") - 1) / (n - 1)


def composite_factor_calculation(X, names, selected, method="zscore"):
    """composite_factor.py:137-218.  Returns [D][A]."""
    if method not in ("zscore", "rank"):
        raise ValueError("method must be 'zscore' or 'rank'")
    pos = [names.index(s) for s in selected]
    sel_names = [names[k] for k in pos]
    F, D, A = X.shape
    adj = X[pos].copy()
    for d in range(D):                                        # :157-178 (per column)
        for suffix, (ql, qh) in SUFFIX.items():
            for j, n in enumerate(sel_names):
                if not n.endswith(suffix):
                    continue
                arr = adj[j, d]
                clean = arr[~np.isnan(arr)]
                if clean.size == 0:
                    adj[j, d] = 0.0
                    continue
                lo, hi = _pct(clean, ql), _pct(clean, qh)
                adj[j, d] = 0.0 if hi == lo else _scale(suffix, arr, lo, hi)
    groups = _prefix_groups(sel_names)
    prox = np.stack([np.stack([_rowmean_skipna(adj[idx, d]) for d in range(D)])
                     for idx in groups.values()])            # [G][D][A]
    comp = np.empty((D, A))
    for d in range(D):
        if method == "zscore":
            z = np.stack([_safe_z(prox[g, d]) for g in range(len(groups))])
            comp[d] = _rowmean_skipna(z)
        else:
            r = np.stack([_rank01(prox[g, d]) for g in range(len(groups))])
            comp[d] = nm.pairwise_sum(np.where(np.isnan(r), 0.0, r).T)   # skipna sum
    mu = nm.nanmean(comp)
    return comp - mu[:, None]


def weighted_composite_factor(X, names, sel_dates_idx, W, method="zscore"):
    """composite_factor.py:220-342.  ``sel_dates_idx[i]`` is the panel date index of
    selection row i (or -1 when the date is not in the panel).  Returns [D][A] with
    non-selected dates 0 (the final reindex().fillna(0))."""
    if method not in ("zscore", "rank"):
        raise ValueError("method must be 'zscore' or 'rank'")
    F, D, A = X.shape
    out = np.zeros((D, A))
    for i, d in enumerate(sel_dates_idx):
        if d < 0:
            continue
        wrow = W[i]
        today = [k for k in range(F) if wrow[k] > 0]
        if not today:
            continue                                          # NaN -> fillna(0)
        tn = [names[k] for k in today]
        adj = X[today, d].copy()                              # [k][A]
        for suffix, (ql, qh) in SUFFIX.items():               # :251-268 pooled
            cols = [j for j, n in enumerate(tn) if n.endswith(suffix)]
            if not cols:
                continue
            vals = adj[cols]
            clean = vals[~np.isnan(vals)]
            if clean.size == 0:
                adj[cols] = 0.0
                continue
            lo, hi = _pct(clean, ql), _pct(clean, qh)
            if lo == hi:
                adj[cols] = 0.0
            else:
                for j in cols:
                    adj[j] = _scale(suffix, adj[j], lo, hi)
        groups = _prefix_groups(tn)
        prox = np.stack([_rowmean_skipna(adj[idx]) for idx in groups.values()])
        gw = [sum(wrow[today[j]] for j in idx) for idx in groups.values()]  # Python sum
        gws = sum(gw)
        if gws > 0:
            gw = [g / gws for g in gw]
        else:
            gw = [1 / len(gw)] * len(gw)
        if method == "zscore":
            normed = [_safe_z(p) for p in prox]
        else:
            normed = [_rank01(p) for p in prox]
        comp = 0
        for g in range(len(normed)):                          # Python sum(): NaN propagates
            comp = comp + normed[g] * gw[g]
        comp = comp - nm.nanmean(np.asarray(comp)[None, :])[0]
        out[d] = np.where(np.isnan(comp), 0.0, comp)
    return out
