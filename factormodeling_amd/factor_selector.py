"""Drop-in replacement for the reference's ``factor_selector.py``.

``single_factor_metrics`` and ``FactorSelector`` keep the reference's signatures,
attributes, logging and outputs (factor_selector.py:26-139).  The per-(factor, date)
Pearson/rank IC and beta loop (two ``pearsonr`` + one ``rankdata`` Python calls per
group in the reference) runs as one ``fmx_ic_daily`` launch over the whole panel, and
the rolling-window metrics of every processed day come from one ``fmx_ic_window``
launch over the daily series.

Rolling selection, dense panels: ``FactorSelector`` shifts factors by one row per symbol
and ``single_factor_metrics`` shifts again inside each window (factor_selector.py:84,
:33), so a window's metrics are the lag-2 daily ICs of its last ``window - 1`` dates.
The device path computes the lag-2 daily series once and summarises windows
[t - W + 1, t).  Ragged panels or a factor_ret_df missing panel dates take the
per-window device path, which recomputes each window exactly as the reference slices it.
"""
from __future__ import annotations

import logging

import numpy as np
import pandas as pd
import torch
from scipy import special

from . import engine
from .factor_selection_methods import (corr_prune_selector, factor_momentum_selector, icir_top_selector,
                                       mvo_selector)
from .panel import device, panel_index
from .profiling import phase

logger = logging.getLogger("factor_selector")

FACTOR_SELECTION_METHODS = {
    "icir_top": icir_top_selector,
    "mvo": mvo_selector,
    "momentum": factor_momentum_selector,
    "corr_prune": corr_prune_selector,
}

METRIC_COLS = ["IC", "IC_IR", "rank_IC", "rank_IC_IR", "factor_return_tstat", "factor_return_pvalue",
               "pct_pos_factor_return"]

# selectors known not to read factors_win / returns_win (no per-day slicing needed)
_NO_PANEL_ARGS = (icir_top_selector, factor_momentum_selector, mvo_selector)


def _metrics_frame(vals: np.ndarray, names) -> pd.DataFrame:
    """[F][8] window summary (device) -> the reference's sorted metrics DataFrame."""
    t = vals[:, 4]
    nb = vals[:, 5]
    with np.errstate(all="ignore"):
        p = np.where(nb > 1, 2.0 * special.stdtr(nb - 1, -np.abs(t)), np.nan)
    df = pd.DataFrame({"factor": list(names), "IC": vals[:, 0], "IC_IR": vals[:, 1], "rank_IC": vals[:, 2],
                       "rank_IC_IR": vals[:, 3], "factor_return_tstat": t, "factor_return_pvalue": p,
                       "pct_pos_factor_return": vals[:, 6]}).set_index("factor")
    return df.sort_values("rank_IC_IR", ascending=False)


def _dense_inputs(factors_df: pd.DataFrame, returns: pd.Series):
    P = panel_index(factors_df.index)
    dev = device()
    with phase("pandas->dense"):
        xv = factors_df.to_numpy(dtype=np.float64, na_value=np.nan)
        r = returns if returns.index.equals(factors_df.index) else returns.reindex(factors_df.index)
        rv = r.to_numpy(dtype=np.float64, na_value=np.nan)
    X = P.to_device(xv, dev)
    R = P.to_device(rv, dev)[0]
    return P, X, R


def _daily(P, X, R, lag: int):
    """Daily stats [4][F][D] of pairs (row-lagged X, R) for one lag."""
    dev = X.device
    pres = P.present(dev)
    if pres is None:
        return engine.ic_daily(X, R, (lag,))[0]
    XL = engine.ts("delay", X, lag, pres)           # row-based lag per symbol
    return engine.ic_daily(XL, R, (0,))[0]


def single_factor_metrics(factors_df: pd.DataFrame, returns: pd.Series) -> pd.DataFrame:
    """factor_selector.py:26-73"""
    names = [c for c in factors_df.columns]
    P, X, R = _dense_inputs(factors_df[names], returns)
    daily = _daily(P, X, R, 1)
    summ = engine.ic_window(daily, [0], [P.D])[0]
    with phase("D2H"):
        summ = summ.cpu().numpy()
    with phase("dense->pandas"):
        return _metrics_frame(summ, names)


class FactorSelector:
    """factor_selector.py:76-139"""

    def __init__(self, factors_df: pd.DataFrame, returns: pd.Series, factor_ret_df: pd.DataFrame, window: int,
                 method: str, method_kwargs: dict = None):
        logger.info(f"Initializing FactorSelector with method='{method}' and window={window}...")
        self._factors_raw = factors_df
        self._factors_lag = None
        self.factor_cols = [c for c in factors_df.columns]
        self.returns = returns
        self.factor_ret_df = factor_ret_df
        self.window = window
        self.method = method
        self.method_kwargs = method_kwargs or {}
        self.factor_selection = None
        # the reference's sorted(set(dates) & set(factor_ret_df.index)) (factor_selector.py:91)
        # on the distinct dates only: a Python set of every (date, symbol) row's Timestamp took
        # 14 s of the 2520 x 5000 drop-in call (profiles/r06/dropin_c2s_*.json)
        fd = pd.Index(factors_df.index.get_level_values("date").unique())
        common = fd.intersection(pd.Index(self.factor_ret_df.index).unique())
        self.dates = sorted(common.tolist())
        logger.info("FactorSelector initialized.")

    @property
    def factors(self) -> pd.DataFrame:
        """``factors_df.groupby(level='symbol').shift(1)`` (computed on the GPU, lazily)."""
        if self._factors_lag is None:
            from .operations import ts_delay
            self._factors_lag = ts_delay(self._factors_raw, 1)
        return self._factors_lag

    @factors.setter
    def factors(self, value):
        self._factors_lag = value

    # ------------------------------------------------------------------------------
    def _contiguous(self, P):
        dpos = P.dates.get_indexer(pd.Index(self.dates))
        return len(dpos) == P.D and bool(np.all(dpos == np.arange(P.D)))

    def _window_metrics(self, P, X, R, proc_idx):
        """[J][F][8] metrics of each processed day's window (device)."""
        W = self.window
        dpos = P.dates.get_indexer(pd.Index(self.dates))
        contiguous = bool(np.all(dpos == np.arange(P.D))) if len(dpos) == P.D else False
        if P.dense and contiguous:
            daily2 = _daily(P, X, R, 2)
            d0 = [i - W + 1 for i in proc_idx]
            d1 = list(proc_idx)
            return engine.ic_window(daily2, d0, d1)
        # general path: rebuild each window exactly as the reference slices it
        dev = X.device
        pres = P.present(dev)
        L1 = engine.ts("delay", X, 1, pres)
        out = []
        for i in proc_idx:
            wd = dpos[max(0, i - W):i]
            Xw = L1[:, wd].contiguous()
            Rw = R[wd].contiguous()
            pw = None if pres is None else pres[wd].contiguous()
            Xw2 = engine.ts("delay", Xw, 1, pw)
            dl = engine.ic_daily(Xw2, Rw, (0,))[0]
            out.append(engine.ic_window(dl, [0], [len(wd)])[0])
        return torch.stack(out) if out else torch.empty((0, X.shape[0], 8), dtype=torch.float64, device=dev)

    def prepare_selection(self) -> pd.DataFrame:
        """factor_selector.py:94-139"""
        if self.factor_selection is not None:
            logger.info("Factor selection already prepared. Returning cached result.")
            return self.factor_selection
        logger.info("Executing rolling factor selection...")
        proc_dates = self.dates[self.window:-1]
        selector_func = FACTOR_SELECTION_METHODS.get(self.method)
        if selector_func is None:
            raise ValueError(f"Unknown factor selection method: {self.method}")
        if not proc_dates:
            self.factor_selection = pd.DataFrame()
            return self.factor_selection
        names = self.factor_cols
        P, X, R = _dense_inputs(self._factors_raw[names], self.returns)
        proc_idx = list(range(self.window, len(self.dates) - 1))
        M = self._window_metrics(P, X, R, proc_idx)                     # [J][F][8] on device
        kw = self.method_kwargs
        device_prune = (selector_func is corr_prune_selector and P.dense and len(names) <= engine.FUSED_GRAM_MAX_F
                        and self._contiguous(P))
        if selector_func is icir_top_selector or device_prune:
            if selector_func is icir_top_selector:
                _, w = engine.select_icir_top(M, kw.get("use_rank_icir", True), kw.get("icir_threshold", 0.03),
                                              kw.get("top_x", 5))
            else:
                # the corr_prune plugin for every day at once: per-date Gram partials of the
                # lag-1 factors pooled per window and the greedy walk on the device
                order, _ = engine.select_icir_top(M, True, -np.inf, len(names))
                _, stats = engine.cs_moment_stats("stats", X)
                s0 = [i - self.window - 1 for i in proc_idx]
                w = engine.corr_prune_windows(X, stats, M, order, self.window, s0, kw.get("use_rank_icir", True),
                                              kw.get("icir_threshold", -np.inf), kw.get("rho", 0.7),
                                              kw.get("top_x", 5))
            with phase("D2H"):
                m0, wh = M[0].cpu().numpy(), w.cpu().numpy()
            with phase("dense->pandas"):
                first = _metrics_frame(m0, names)
                cols = list(first.index)
                pos = [names.index(c) for c in cols]
                sel = pd.DataFrame(wh[:, pos], index=pd.Index(proc_dates), columns=cols)
        else:
            Mh = M.cpu().numpy()
            vecs = []
            for j, today in enumerate(proc_dates):
                i = proc_idx[j]
                window_dates = self.dates[max(0, i - self.window):i]
                metrics_df = _metrics_frame(Mh[j], names)
                factor_ret_win = self.factor_ret_df.loc[window_dates].copy()
                if selector_func in _NO_PANEL_ARGS:
                    factors_win = returns_win = None
                else:
                    factors_win = self.factors.loc[window_dates].copy()
                    returns_win = self.returns.loc[window_dates].copy()
                vec = selector_func(metrics_df, factors_win, returns_win, factor_ret_win, today, window_dates, **kw)
                vec.name = today
                vecs.append(vec)
            sel = pd.concat(vecs, axis=1).T
        selection_df = sel
        selection_df.index.name = "date"
        selection_df.columns.name = "factor"
        selection_df = selection_df.div(selection_df.sum(axis=1), axis=0).fillna(0)
        self.factor_selection = selection_df
        return selection_df
