"""multi_manager.compute_multimanager_weights on the GPU.

Reference: multi_manager.py:32-81.  Each factor is a manager whose book is
Simulation._daily_trade_list over ``factors_df[fac].dropna()`` with the settings' method
('equal' or 'linear'); all managers' books come from ONE batched launch (``fmx_trade_books``,
NaN cells = no row), and each weight date folds the managers' books and counts in
``factor_weights`` column order (``k_mm_combine``).  Returns the reference's
``(final_weights, final_counts)``: nonzero weights over ``(date, symbol)``, counts indexed
by date.  'mvo' / 'mvo_turnover' managers (a host QP per date) take their books from
``compute_manager_weights`` -- the drop-in ``Simulation._daily_trade_list``, which hands
them to the reference's own solvers -- and fold on the device like the others.  Columns
absent from ``factors_df`` log the reference's warning (:42-44).  Symbol order within a date: ``daily_weights.add(mgr_w_today * fac_w,
fill_value=0)`` (:63) aligns the first-appearance ``all_symbols`` index with a manager's
date-sorted book index; unless the two are identical pandas returns their sorted union,
and a date without any contribution holds only zeros (dropped by ``!= 0``), so the
surviving weights of every date are in sorted symbol order.
"""
from __future__ import annotations

import logging

import numpy as np
import pandas as pd
import torch

from . import engine as E
from .panel import device, panel_index
from .simulation import by_date, trade_books

logger = logging.getLogger("multi_manager")
HOST_METHODS = ("mvo", "mvo_turnover")


def _setting(settings, key, default):
    if isinstance(settings, dict):
        return settings.get(key, default)
    return getattr(settings, key, default)


def _host_books(pi, factors_df, mgrs, settings, dev):
    """Books of host-solved managers (multi_manager.py:45-48): each factor's
    ``dropna()`` series through ``compute_manager_weights``, scattered onto the panel grid
    ([F][D][A] shifted weights, NaN = no row; [F][D][2] counts, NaN = no book that date)."""
    F, D, A = len(mgrs), pi.D, pi.A
    Wf = np.full((F, D, A), np.nan)
    cnt = np.full((F, D, 2), np.nan)
    for f, fac in enumerate(mgrs):
        w, c = compute_manager_weights(factors_df[fac].dropna(), settings, name=fac)
        if len(w):
            d = pi.dates.get_indexer(w.index.get_level_values(0))
            a = pi.symbols.get_indexer(w.index.get_level_values(1))
            Wf[f, d, a] = w.to_numpy(dtype=np.float64, na_value=np.nan)
        if len(c):
            cnt[f, pi.dates.get_indexer(c.index)] = c[["long_count", "short_count"]].to_numpy(dtype=np.float64)
    return torch.as_tensor(Wf, device=dev), torch.as_tensor(cnt, device=dev)


def compute_multimanager_weights(factors_df: pd.DataFrame, factor_weights: pd.DataFrame, settings):
    method = _setting(settings, "method", "equal")
    pct = float(_setting(settings, "pct", 0.1))
    max_weight = float(_setting(settings, "max_weight", 0.03))
    mgrs = []
    for fac in factor_weights.columns:
        if fac not in factors_df.columns:
            logger.warning(f"Factor {fac} not in factors_df, skipping.")
            continue
        if fac not in mgrs:
            mgrs.append(fac)
    if mgrs and method not in ("equal", "linear") + HOST_METHODS:
        raise ValueError(f"Unknown method {method}")
    all_symbols = factors_df.index.get_level_values("symbol").unique()
    if len(factor_weights.index) == 0:
        return pd.Series(dtype=float), pd.DataFrame(columns=["long_count", "short_count"])
    factors_df = by_date(factors_df)
    pi = panel_index(factors_df.index)
    dev = device()
    F, D, A = len(mgrs), pi.D, pi.A
    if F and method in HOST_METHODS:
        Wf, cnt = _host_books(pi, factors_df, mgrs, settings, dev)
    elif F:
        Wf, cnt = trade_books(pi, factors_df[mgrs].to_numpy(dtype=np.float64), method, pct, max_weight, True)
    else:
        Wf = torch.empty((1, D, A), dtype=torch.float64, device=dev)
        cnt = torch.full((1, D, 2), float("nan"), dtype=torch.float64, device=dev)
    colmap = [mgrs.index(c) if c in mgrs else -1 for c in factor_weights.columns]
    wdate = pi.dates.get_indexer(factor_weights.index)
    out, oc = E.mm_combine(Wf, cnt, factor_weights.to_numpy(dtype=np.float64), colmap, wdate)
    perm = pi.symbols.get_indexer(all_symbols.sort_values())
    out = out.cpu().numpy()[:, perm]
    oc = oc.cpu().numpy()
    index = pd.MultiIndex.from_product([factor_weights.index, all_symbols.sort_values()], names=["date", "symbol"])
    final = pd.Series(out.reshape(-1), index=index)
    final = final[final != 0]
    counts = pd.DataFrame({"long_count": oc[:, 0], "short_count": oc[:, 1]},
                          index=pd.Index(factor_weights.index, name="date"))
    return final, counts


def compute_manager_weights(factor_series, settings, name="manager"):
    """multi_manager.py:15-29: one manager's book through Simulation._daily_trade_list."""
    from .portfolio_simulation import Simulation, SimulationSettings
    sim_settings = settings if isinstance(settings, SimulationSettings) else SimulationSettings(**settings)
    sim = Simulation(name=name, custom_feature=factor_series, settings=sim_settings)
    return sim._daily_trade_list()


def run_multimanager_backtest(factors_df, returns, cap_flag, factor_weights, settings):
    """multi_manager.py:84-100: combined book -> Simulation._daily_portfolio_returns (device)."""
    from .portfolio_simulation import Simulation, SimulationSettings
    weights, counts = compute_multimanager_weights(factors_df, factor_weights, settings)
    sim_settings = settings if isinstance(settings, SimulationSettings) else SimulationSettings(**settings)
    sim = Simulation(name="multimanager", custom_feature=weights, settings=sim_settings)
    result, top_longs, top_shorts = sim._daily_portfolio_returns(weights)
    return result, top_longs, top_shorts, counts
