"""Oracle restatement of factor_selector.py / factor_selection_methods.py.

Test infrastructure only (see oracle/__init__.py).

Inputs are dense: ``X[F][D][A]`` exposures, ``R[D][A]`` returns, optional
``present[D][A]``.  The daily statistics restate the reference's per-(factor, date)
loop (factor_selector.py:36-48) with scipy's ``pearsonr``/``rankdata`` formulas
(scipy 1.15.3 ``_stats_py.py:4272``/``:10108``) and the per-factor summary
(:50-59) with numpy ``mean``/``std(ddof=1)`` and scipy ``ttest_1samp``.
"""
from __future__ import annotations

import numpy as np
from scipy import special

from . import numerics as nm
from . import ops

COLS = ["IC", "IC_IR", "rank_IC", "rank_IC_IR", "factor_return_tstat",
        "factor_return_pvalue", "pct_pos_factor_return"]


def pearsonr(x, y):
    """scipy.stats.pearsonr statistic (1-D, n >= 3): two-pass, max-scaled norms,
    clipped to [-1, 1], NaN when either input is exactly constant."""
    if np.all(x == x[0]) or np.all(y == y[0]):
        return np.nan
    xm = x - nm.np_mean(x)
    ym = y - nm.np_mean(y)
    xmax = np.max(np.abs(xm))
    ymax = np.max(np.abs(ym))
    nx = xmax * np.sqrt(np.dot(xm / xmax, xm / xmax))
    ny = ymax * np.sqrt(np.dot(ym / ymax, ym / ymax))
    r = nm.pairwise_sum(xm / nx * ym / ny)
    return float(np.clip(r, -1.0, 1.0))


def rankdata(x):
    """scipy.stats.rankdata(method='average') for NaN-free input."""
    return nm.rank_1d(x, "average")


def daily_stats(f, r):
    """factor_selector.py:37-48 for one date: (n, IC, rank_IC, beta|NaN)."""
    ok = ~np.isnan(f) & ~np.isnan(r)
    f, r = f[ok], r[ok]
    n = len(f)
    if n < 3:
        return n, np.nan, np.nan, np.nan
    ic = pearsonr(f, r)
    ric = pearsonr(rankdata(f), r)
    den = np.dot(f, f)
    beta = np.dot(f, r) / den if den > 0 else np.nan
    return n, ic, ric, beta


def lag_panel(X, lag, present=None):
    """``groupby(level='symbol').shift(lag)`` (row-based) for every factor."""
    return np.stack([ops.ts_delay(X[k], lag, present) for k in range(X.shape[0])])


def summarize(ic, ric, beta):
    """factor_selector.py:50-59 from the per-date lists (already n>=3 filtered)."""
    ic = np.asarray(ic, dtype=np.float64); ic = ic[~np.isnan(ic)]
    ric = np.asarray(ric, dtype=np.float64); ric = ric[~np.isnan(ric)]
    beta = np.asarray(beta, dtype=np.float64); beta = beta[~np.isnan(beta)]
    ic_mean = nm.np_mean(ic) if ic.size else np.nan
    ic_ir = ic_mean / nm.np_std_ddof1(ic) if ic.size > 1 else np.nan
    r_mean = nm.np_mean(ric) if ric.size else np.nan
    r_ir = r_mean / nm.np_std_ddof1(ric) if ric.size > 1 else np.nan
    if beta.size > 1:
        n = beta.size
        m = nm.np_mean(beta)
        v = nm.np_mean((beta - m) ** 2) * (n / (n - 1))
        with np.errstate(all="ignore"):
            t = m / np.sqrt(v / n)
        p = 2 * special.stdtr(n - 1, -np.abs(t))
    else:
        t = p = np.nan
    pct = np.mean(beta > 0) if beta.size else np.nan
    return [ic_mean, ic_ir, r_mean, r_ir, t, p, pct]


def nargsort_desc(v):
    """pandas ``sort_values(ascending=False)`` order: NaN last, ties by position
    (the reference's F is small enough that numpy's argsort is stable)."""
    v = np.asarray(v, dtype=np.float64)
    idx = np.arange(len(v))
    m = np.isnan(v)
    nn, ni = v[~m][::-1], idx[~m][::-1]
    order = ni[np.argsort(nn, kind="stable")][::-1]
    return np.concatenate([order, idx[m]])


def single_factor_metrics(X, R, present=None, shifted=None):
    """factor_selector.py:26-73.  Returns (order, vals[F][7]) where ``order`` sorts
    factors by rank_IC_IR descending (NaN last)."""
    F, D, A = X.shape
    S = lag_panel(X, 1, present) if shifted is None else shifted
    rows = []
    for k in range(F):
        ic, ric, beta = [], [], []
        for t in range(D):
            idx = np.arange(A) if present is None else np.nonzero(present[t])[0]
            n, a, b, c = daily_stats(S[k, t, idx], R[t, idx])
            if n < 3:
                continue
            ic.append(a); ric.append(b)
            if not np.isnan(c):
                beta.append(c)
        rows.append(summarize(ic, ric, beta))
    vals = np.array(rows, dtype=np.float64)
    order = nargsort_desc(vals[:, 3])
    return order, vals


# --------------------------------------------------------------------------- selectors
def icir_top(order, vals, icir_threshold=0.03, top_x=5, use_rank_icir=True, **kw):
    """factor_selection_methods.py:6-26 -- returns weights aligned to ``order``."""
    col = 3 if use_rank_icir else 1
    v = vals[order, col]
    with np.errstate(invalid="ignore"):
        keep = np.nonzero(v > icir_threshold)[0]
    # nlargest(keep='first'): largest values, ties by position in the sorted frame
    sel = keep[np.argsort(-v[keep], kind="stable")][:top_x]
    w = np.zeros(len(order))
    w[sel] = 1.0
    if w.sum() > 0:
        w = w / w.sum()
    return w


def momentum(order, fret_win, max_weight=1.0, **kw):
    """factor_selection_methods.py:28-58 -- weights aligned to ``order``.
    ``fret_win`` is ``[W][F]`` in original column order."""
    fw = np.ascontiguousarray(np.asarray(fret_win, dtype=np.float64)[:, order].T)  # [F][W]
    mom = nm.pairwise_sum(fw)
    mom = np.where(mom < 0, 0.0, mom)
    if max_weight < 1.0:
        mom = np.where(mom > max_weight, max_weight, mom)
    s = nm.pairwise_sum(mom[None, :])[0]
    if s > 0:
        return mom / s
    return np.zeros(len(order))


def corr_prune(order, vals, Xw, rho=0.7, top_x=5, icir_threshold=-np.inf, use_rank_icir=True, **kw):
    """Builder-defined corr_prune plugin (parity unpinned by the reference):
    factors in metrics order above ``icir_threshold``, greedy-pruned on the correlation of
    the window's per-date z-scored (lag-1) exposures, equal weights.  Weights aligned to
    ``order``."""
    from . import gram
    col = 3 if use_rank_icir else 1
    C = gram.corr_matrix(Xw[order])
    v = vals[order, col]
    with np.errstate(invalid="ignore"):
        cand = [i for i in range(len(order)) if v[i] > icir_threshold]
    kept = gram.greedy_prune(C, cand, rho, top_x)
    w = np.zeros(len(order))
    if kept:
        w[kept] = 1.0 / len(kept)
    return w


def factor_selector(X, R, FR, fr_dates_mask, window, method, method_kwargs=None, present=None):
    """factor_selector.py:76-139 on a panel whose date axis is the full sorted date
    list.  ``fr_dates_mask[d]`` says whether date d is in factor_ret_df's index.
    Returns (row_dates_idx, col_order, W[rows][F]) -- W before row normalisation is
    applied as the reference does (div by row sum, fillna(0)).
    """
    kw = dict(method_kwargs or {})
    F, D, A = X.shape
    L1 = lag_panel(X, 1, present)                           # self.factors (lag #1)
    dates = [d for d in range(D) if fr_dates_mask[d]]
    proc = dates[window:-1]
    cols = None
    vecs = []
    for today in proc:
        idx = dates.index(today)
        wd = dates[max(0, idx - window):idx]
        # window slice, then single_factor_metrics shifts again within the slice
        Xw = L1[:, wd]
        Rw = R[wd]
        Pw = None if present is None else present[wd]
        order, vals = single_factor_metrics(Xw, Rw, Pw)
        if method == "icir_top":
            w = icir_top(order, vals, **kw)
        elif method == "momentum":
            w = momentum(order, FR[wd], **kw)
        elif method == "corr_prune":
            w = corr_prune(order, vals, Xw, **kw)
        else:
            raise ValueError(f"Unknown factor selection method: {method}")
        if cols is None:
            cols = list(order)
        vec = np.zeros(F)
        vec[order] = w
        vecs.append(vec[cols])
    if not vecs:
        return [], [], np.zeros((0, F))
    Wm = np.array(vecs)
    s = nm.pairwise_sum(Wm)
    with np.errstate(all="ignore"):
        Wn = Wm / s[:, None]
    Wn = np.where(np.isnan(Wn), 0.0, Wn)
    return proc, cols, Wn
