"""Drop-in replacement for the reference's ``composite_factor.py``.

``composite_factor_calculation`` (composite_factor.py:137-218) and
``weighted_composite_factor`` (:220-342) keep their signatures and outputs (Series named
``composite_factor`` on ``factors_df.index``); the per-date percentiles, suffix scaling,
prefix-group proxies, z-score / rank normalisation, weighting and demeaning run in the
gfx950 kernels of ``csrc/composite.hip`` and ``csrc/cs_ops.hip``.  The two plotting helpers
the notebook imports (pipeline.ipynb:55) are host-side matplotlib code, as in the
reference.
"""
from __future__ import annotations

import math

import numpy as np
import pandas as pd
import torch

from . import engine
from .panel import device, panel_index
from .profiling import phase


def _prefix_groups(names):
    groups = {}
    for k, n in enumerate(names):
        groups.setdefault(n.split("_", 1)[0], []).append(k)
    return groups


def composite_factor_calculation(factors_df: pd.DataFrame, selected_factors: list, method: str = "zscore"):
    """composite_factor.py:137-218"""
    if method not in ("zscore", "rank"):
        raise ValueError("method must be 'zscore' or 'rank'")
    pos = list(selected_factors)
    P = panel_index(factors_df.index)
    dev = device()
    X = P.to_device(factors_df[pos].to_numpy(dtype=np.float64, na_value=np.nan), dev)
    pres = P.present(dev)
    Adj = engine.comp_adj(X, list(range(len(pos))), [engine.suffix_code(n) for n in pos])
    if pres is not None:
        Adj.masked_fill_(pres.unsqueeze(0) == 0, float("nan"))
    groups = list(_prefix_groups(pos).values())
    Prox = engine.comp_proxy(Adj, groups)
    if method == "zscore":
        Nrm = engine.cs_moment("market_neutralize", Prox, pres)   # safe_zcol == market_neutralize
        comp = engine.comp_combine(Nrm, 0, pres)
    else:
        Nrm = engine.cs_rank(Prox, "scipy_average", pres)
        comp = engine.comp_combine(Nrm, 1, pres)
    vals = P.from_device(comp.unsqueeze(0))[:, 0]
    return pd.Series(vals, index=factors_df.index, name="composite_factor")


def weighted_plan(pdate, W, names):
    """Per selection row j (panel date index pdate[j], -1 = not a panel date; weights
    W[j] over ``names`` in selection_df column order): the selected columns (w > 0, column
    order), their suffix codes, prefix groups numbered by first appearance among them,
    the group weights (composite_factor.py:276-290: sums in column order, normalised, or
    equal when all zero) and the pooled suffix column lists (:251-268)."""
    W = np.asarray(W, dtype=np.float64)
    J, F = W.shape
    suffix = np.array([engine.suffix_code(n) for n in names], dtype=np.int32)
    _, pid = np.unique(np.array([n.split("_", 1)[0] for n in names], dtype=object).astype(str),
                       return_inverse=True)
    P = int(pid.max()) + 1 if F else 1
    sel = W > 0
    KMAX = int(max(1, sel.sum(axis=1).max() if J else 1))
    sel &= (np.asarray(pdate) >= 0)[:, None]
    col = np.zeros((J, KMAX), np.int32)
    suf = np.zeros((J, KMAX), np.int32)
    grp = np.full((J, KMAX), -1, np.int32)
    gwa = np.zeros((J, KMAX), np.float64)
    ncol = sel.sum(axis=1).astype(np.int32)
    pd_out = np.where(ncol > 0, np.asarray(pdate), -1).astype(np.int32)
    # selected entries in row-major order = each row's columns in column order
    jj, cc = np.nonzero(sel)
    kk = np.arange(jj.size) - np.concatenate([[0], np.cumsum(ncol)])[jj]
    col[jj, kk] = cc
    suf[jj, kk] = suffix[cc]
    # prefix groups numbered by first appearance within the row
    key = jj.astype(np.int64) * P + pid[cc]
    uk, first, inv = np.unique(key, return_index=True, return_inverse=True)
    order = np.argsort(first, kind="stable")           # unique groups in (row, first position) order
    urow = (uk // P)[order]
    starts = np.flatnonzero(np.r_[True, urow[1:] != urow[:-1]]) if urow.size else np.zeros(0, np.int64)
    run = np.repeat(starts, np.diff(np.r_[starts, urow.size]))
    gnum = np.empty(uk.size, np.int64)
    gnum[order] = np.arange(urow.size) - run
    grp[jj, kk] = gnum[inv]
    ngrp = np.bincount(uk // P, minlength=J).astype(np.int32) if uk.size else np.zeros(J, np.int32)
    # group sums (composite_factor.py:281: pandas Series.sum = numpy sum over the members in
    # column order: sequential from 0 below 8 members, numpy's pairwise sum from 8)
    vals = W[jj, cc]
    gsum = np.zeros(uk.size)
    np.add.at(gsum, inv, vals)
    big = np.flatnonzero(np.bincount(inv, minlength=uk.size) >= 8)
    for u in big:
        gsum[u] = vals[inv == u].sum()
    tot = np.zeros(J)                                   # Python sum over groups in order (:282)
    np.add.at(tot, urow, gsum[order])
    r = uk // P
    gw = np.where(tot[r] > 0, gsum / np.where(tot[r] > 0, tot[r], 1.0), 1.0 / np.maximum(ngrp[r], 1))
    gwa[r, gnum] = gw
    # pooled suffix column lists per (row, suffix 1..4), columns in column order (:251-268)
    sc = suffix[cc]
    m = (sc >= 1) & (sc <= 4)
    idx = np.flatnonzero(m)
    idx = idx[np.lexsort((kk[idx], sc[idx], jj[idx]))]
    scol = cc[idx].astype(np.int32)
    cnt = np.bincount(jj[m] * 4 + (sc[m] - 1), minlength=4 * J) if J else np.zeros(0, np.int64)
    soff = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int32)
    return {"pdate": pd_out, "ncol": ncol, "col": col, "suf": suf, "grp": grp, "ngrp": ngrp, "gw": gwa,
            "KMAX": KMAX, "soff": soff, "scol": scol if scol.size else np.zeros(1, np.int32)}


def _weighted_plan(P, selection_df: pd.DataFrame, used: list):
    """weighted_plan for a selection DataFrame restricted to the ``used`` columns."""
    pdate = P.dates.get_indexer(selection_df.index) if len(P.dates) else np.full(len(selection_df), -1)
    W = selection_df[used].to_numpy(dtype=np.float64) if used else np.zeros((len(selection_df), 0))
    return weighted_plan(pdate, W, used)


def weighted_composite_factor(factors_df: pd.DataFrame, selection_df: pd.DataFrame, method: str = "zscore") -> pd.Series:
    """composite_factor.py:220-342"""
    if method not in ("zscore", "rank"):
        raise ValueError("method must be 'zscore' or 'rank'")
    if len(selection_df) == 0:
        raise ValueError("No objects to concatenate")
    used = [c for c in selection_df.columns if (selection_df[c] > 0).any()]
    P = panel_index(factors_df.index)
    dev = device()
    if used:
        with phase("pandas->dense"):
            xv = factors_df[used].to_numpy(dtype=np.float64, na_value=np.nan)
        X = P.to_device(xv, dev)
    else:
        X = torch.zeros((1, P.D, P.A), dtype=torch.float64, device=dev)
    with phase("host plan"):
        plan = _weighted_plan(P, selection_df, used)
    out = engine.wcomp(X, plan, method, P.present(dev))
    vals = P.from_device(out.unsqueeze(0))[:, 0]
    return pd.Series(vals, index=factors_df.index, name="composite_factor")


# ----------------------------------------------------------------------------- plotting (host)
def plot_factor_distributions(factors_df: pd.DataFrame, exclude: list = None, bins: int = 50, ncols: int = 3,
                              figsize: tuple = (15, 5)):
    """composite_factor.py:17-44 -- histogram grid of factor columns (host matplotlib)."""
    import matplotlib.pyplot as plt
    exclude = exclude or []
    cols = [c for c in factors_df.columns if c not in exclude]
    nrows = max(1, math.ceil(len(cols) / ncols))
    fig, axes = plt.subplots(nrows, ncols, figsize=(figsize[0], figsize[1] * nrows), squeeze=False)
    flat = axes.ravel()
    for ax, c in zip(flat, cols):
        ax.hist(factors_df[c].dropna(), bins=bins, density=True, alpha=0.7)
        ax.set_title(c)
        ax.set_xlabel("Value")
        ax.set_ylabel("Density")
    for ax in flat[len(cols):]:
        ax.axis("off")
    plt.tight_layout()
    plt.show()


def plot_quantile_backtests_log(com_factors_df: pd.DataFrame, returns: pd.Series, n_groups: int = 5, ncols: int = 2,
                                figsize: tuple = (20, 6)):
    """composite_factor.py:47-134 -- per-date quantile buckets (1 = top), lagged one row
    per symbol, mean log return per bucket, cumulative P&L and the L1-S{n} spread."""
    import matplotlib.pyplot as plt

    def buckets(feature: pd.Series) -> pd.DataFrame:
        lbl = feature.groupby(level="date").transform(
            lambda x: pd.qcut(x.rank(method="first"), n_groups, labels=False, duplicates="drop"))
        q = (n_groups - lbl).astype("Int64").groupby(level="symbol").shift(1)
        df = pd.DataFrame({"log_ret": returns, "group": q}).dropna(subset=["group", "log_ret"])
        g = df.reset_index().groupby(["date", "group"])["log_ret"].mean().unstack(level="group").sort_index()
        return g.reindex(columns=range(1, n_groups + 1))

    facs = list(com_factors_df.columns)
    nrows = max(1, math.ceil(len(facs) / ncols))
    fig, axes = plt.subplots(nrows, ncols, figsize=(figsize[0], figsize[1] * nrows), squeeze=False)
    for i, fac in enumerate(facs):
        ax = axes[i // ncols][i % ncols]
        g = buckets(com_factors_df[fac])
        cum = np.expm1(g.cumsum())
        cum[f"DN_L1-S{n_groups}"] = np.expm1((g[1] - g[n_groups]).cumsum())
        for line in cum.columns:
            if str(line).startswith("DN_L1-S"):
                ax.plot(cum.index, cum[line], label=line, color="black", linewidth=2)
            else:
                ax.plot(cum.index, cum[line], label=line)
        ax.set_title(fac)
        ax.set_xlabel("Date")
        ax.set_ylabel("Cumulative Return")
        ax.legend(loc="upper left", fontsize="small")
        ax.grid(True)
    for k in range(len(facs), nrows * ncols):
        fig.delaxes(axes[k // ncols][k % ncols])
    plt.tight_layout()
    plt.show()
