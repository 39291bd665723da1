"""Drop-in replacement for the reference's ``factor_selection_methods.py``.

The selector functions keep the reference's plugin signature
``f(metrics_df, factors_win, returns_win, factor_ret_win, today, window, **kwargs) ->
pd.Series`` (factor_selection_methods.py:6, :28, :119) so user code and the
``FACTOR_SELECTION_METHODS`` registry keep working.  They are O(F) host functions; the
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
    """factor_selection_methods.py:6-26"""
    col = "rank_IC_IR" if use_rank_icir else "IC_IR"
    selected = metrics_df[metrics_df[col] > icir_threshold].nlargest(top_x, col)
    vec = pd.Series(0.0, index=metrics_df.index, name=today)
    vec.loc[selected.index] = 1.0
    if vec.sum() > 0:
        vec = vec / vec.sum()
    return vec


def factor_momentum_selector(metrics_df, factors_win, returns_win, factor_ret_win, today, window, max_weight=1.0,
                             **kwargs):
    """factor_selection_methods.py:28-58"""
    factor_names = metrics_df.index.tolist()
    momentum = factor_ret_win.loc[:, factor_names].sum()
    momentum = momentum.clip(lower=0)
    if max_weight < 1.0:
        momentum = momentum.clip(upper=max_weight)
    vec = pd.Series(0.0, index=momentum.index, name=today)
    if momentum.sum() > 0:
        vec = momentum / momentum.sum()
    return vec


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
    target = mean_corr * np.outer(std, std)
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
    """factor_selection_methods.py:119-175.  Host-side QP (out of the GPU scope); needs
    cvxpy exactly like the reference."""
    try:
        import cvxpy as cp
    except ImportError as e:  # pragma: no cover - cvxpy is absent in this image
        raise ImportError("mvo_selector needs cvxpy (host QP solver), as in the reference") from e
    factor_names = metrics_df.index.tolist()
    n = len(factor_names)
    mean = factor_ret_win[factor_names].mean()
    if use_shrinkage:
        cov = pd.DataFrame(ledoit_wolf_shrinkage(factor_ret_win[factor_names].values), index=factor_names,
                           columns=factor_names)
    else:
        cov = factor_ret_win[factor_names].cov()
    w = cp.Variable(n)
    cov_matrix = 0.5 * (cov.values + cov.values.T)
    obj = mean.values @ w - risk_aversion * cp.quad_form(w, cov_matrix)
    if turnover_penalty > 0 and previous_weights is not None:
        prev = previous_weights.reindex(factor_names).fillna(0).values
        obj = obj - turnover_penalty * cp.norm1(w - prev)
    constraints = [cp.sum(w) == 1, w >= 0, w <= (max_weight if max_weight < 1.0 else 1)]
    prob = cp.Problem(cp.Maximize(obj), constraints)
    try:
        prob.solve()
        weights = w.value
        if weights is None:
            weights = np.zeros(n)
    except Exception:
        weights = np.zeros(n)
    vec = pd.Series(weights, index=factor_names, name=today)
    if vec.sum() > 0:
        vec = vec / vec.sum()
    return vec


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
