"""Drop-in replacement for the reference's ``factor_selection_methods.py``.

The selector functions keep the reference's plugin signature
``f(metrics_df, factors_win, returns_win, factor_ret_win, today, window, **kwargs) ->
pd.Series`` (factor_selection_methods.py:6, :28, :119) so user code and the
``FACTOR_SELECTION_METHODS`` registry keep working.  icir_top and momentum are O(F) numpy
functions; mvo (a cvxpy QP) is the reference's own selector, loaded by path.  The
O(D x A x F) work they consume (window metrics) is computed on the GPU by
``factor_selector``, which also runs ``icir_top`` fully on the device when the registry
entry is the built-in one.

``corr_prune_selector`` is builder-defined (no reference counterpart): it
prunes the ICIR ranking greedily by the fp64-MFMA factor-correlation matrix.
"""
from __future__ import annotations

import numpy as np
import pandas as pd


def icir_top_selector(metrics_df, factors_win, returns_win, factor_ret_win, today, window, icir_threshold=0.03,
                      top_x=5, use_rank_icir=True, **kwargs):
    """Equal weights on the ``top_x`` factors whose (rank_)IC_IR exceeds ``icir_threshold``
    (factor_selection_methods.py:6-26: ``nlargest`` over the thresholded frame, ties kept in
    frame order -- a stable descending argsort here).  The pipeline's day-by-day selection
    runs the same rule on the device (``k_select_icir_top``)."""
    col = "rank_IC_IR" if use_rank_icir else "IC_IR"
    v = metrics_df[col].to_numpy(dtype=np.float64)
    with np.errstate(invalid="ignore"):
        cand = np.flatnonzero(v > icir_threshold)              # NaN never passes
    sel = cand[np.argsort(-v[cand], kind="stable")][:max(int(top_x), 0)]
    w = np.zeros(len(v))
    if sel.size:
        w[sel] = 1.0 / sel.size
    return pd.Series(w, index=metrics_df.index, name=today)


def factor_momentum_selector(metrics_df, factors_win, returns_win, factor_ret_win, today, window, max_weight=1.0,
                             **kwargs):
    """Weights proportional to each factor's positive window return sum, optionally capped
    at ``max_weight`` (factor_selection_methods.py:28-58).  The per-factor sums run over the
    factor-major copy of the window (NaN -> 0), the same pairwise order as the reference's
    column sums."""
    names = metrics_df.index.tolist()
    fw = np.ascontiguousarray(factor_ret_win.loc[:, names].to_numpy(dtype=np.float64, na_value=np.nan).T)
    mom = np.where(np.isnan(fw), 0.0, fw).sum(axis=1)
    mom = np.maximum(mom, 0.0)
    if max_weight < 1.0:
        mom = np.minimum(mom, max_weight)
    tot = mom.sum()
    if tot > 0:                                  # (the reference's quotient Series is unnamed)
        return pd.Series(mom / tot, index=pd.Index(names))
    return pd.Series(np.zeros(len(names)), index=pd.Index(names), name=today)


def ledoit_wolf_shrinkage(returns):
    """factor_selection_methods.py:60-117 (constant-correlation target), vectorised."""
    returns = np.asarray(returns, dtype=np.float64)
    n, p = returns.shape
    sample_cov = np.cov(returns, rowvar=False)
    var = np.diag(sample_cov)
    std = np.sqrt(var)
    iu = np.triu_indices(p, 1)
    ok = (std[iu[0]] > 0) & (std[iu[1]] > 0)
    corr = sample_cov[iu][ok] / (std[iu[0]][ok] * std[iu[1]][ok])
    mean_corr = np.mean(corr) if corr.size else 0
    target = (mean_corr * std)[:, None] * std[None, :]      # (mean_corr * std_i) * std_j, as the loop
    np.fill_diagonal(target, var)
    d = np.sum((sample_cov - target) ** 2)
    rc = returns - returns.mean(axis=0)
    cov_factors = np.zeros((p, p))
    for k in range(n):
        cov_factors += (np.outer(rc[k], rc[k]) - sample_cov) ** 2
    cov_factors /= n
    lam = max(0, min(1, np.sum(cov_factors) / d))
    return lam * target + (1 - lam) * sample_cov


def mvo_selector(metrics_df, factors_win, returns_win, factor_ret_win, today, window, risk_aversion=1.0,
                 max_weight=1.0, turnover_penalty=0.0, previous_weights=None, use_shrinkage=True, **kwargs):
    """Mean-variance factor weights (factor_selection_methods.py:119-175): a host cvxpy QP,
    outside the GPU scope.  Handed to the reference's own selector, loaded by path from
    ``$FMX_REFERENCE_DIR`` (``_refload``, as the drop-in ``Simulation`` does for its MVO
    methods), so the solver setup is the reference's exactly; it needs cvxpy like the
    reference."""
    from . import _refload
    mod = _refload.load("factor_selection_methods.py", "mvo_selector")
    return mod.mvo_selector(metrics_df, factors_win, returns_win, factor_ret_win, today, window,
                                 risk_aversion=risk_aversion, max_weight=max_weight,
                                 turnover_penalty=turnover_penalty, previous_weights=previous_weights,
                                 use_shrinkage=use_shrinkage, **kwargs)


def corr_prune_selector(metrics_df, factors_win, returns_win, factor_ret_win, today, window, rho=0.7, top_x=5,
                        icir_threshold=-np.inf, use_rank_icir=True, **kwargs):
    """Builder-defined (parity unpinned by the reference): walk factors by
    (rank_)IC_IR descending, skip those at or below ``icir_threshold``, keep a factor iff
    its |correlation| with every kept factor is < ``rho`` (correlation of per-date
    z-scored exposures over the window, fp64 MFMA Gram), stop at ``top_x``; equal
    weights."""
    from . import engine
    from .panel import device, panel_index
    col = "rank_IC_IR" if use_rank_icir else "IC_IR"
    names = list(metrics_df.index)
    vec = pd.Series(0.0, index=metrics_df.index, name=today)
    if factors_win is None or len(factors_win) == 0:
        return vec
    P = panel_index(factors_win.index)
    dev = device()
    X = P.to_device(factors_win[names].to_numpy(dtype=np.float64, na_value=np.nan), dev)
    C = engine.corr_matrix(X)
    vals = metrics_df[col].to_numpy(dtype=np.float64)
    cand = [i for i in range(len(names)) if vals[i] > icir_threshold]
    kept = engine.greedy_prune(C, cand, rho=rho, top_x=top_x)
    if kept:
        vec.iloc[kept] = 1.0 / len(kept)
    return vec
