"""multi_manager.compute_multimanager_weights on the GPU.

Reference: multi_manager.py:32-81.  Each factor is a manager whose book is
Simulation._daily_trade_list over ``factors_df[fac].dropna()`` with the settings' method
('equal' or 'linear'); all managers' books come from ONE batched launch (``fmx_trade_books``,
NaN cells = no row), and each weight date folds the managers' books and counts in
``factor_weights`` column order (``k_mm_combine``).  Returns the reference's
``(final_weights, final_counts)``: nonzero weights over ``(date, symbol)``, counts indexed
by date.  Symbol order within a date: ``daily_weights.add(mgr_w_today * fac_w,
fill_value=0)`` (:63) aligns the first-appearance ``all_symbols`` index with a manager's
date-sorted book index; unless the two are identical pandas returns their sorted union,
and a date without any contribution holds only zeros (dropped by ``!= 0``), so the
surviving weights of every date are in sorted symbol order.
"""
from __future__ import annotations

import numpy as np
import pandas as pd
import torch

from . import engine as E
from .panel import device, panel_index
from .simulation import by_date, trade_books


def _setting(settings, key, default):
    if isinstance(settings, dict):
        return settings.get(key, default)
    return getattr(settings, key, default)


def compute_multimanager_weights(factors_df: pd.DataFrame, factor_weights: pd.DataFrame, settings):
    method = _setting(settings, "method", "equal")
    if method not in ("equal", "linear"):
        raise NotImplementedError(f"method {method!r}: the device runs 'equal' and 'linear' managers")
    pct = float(_setting(settings, "pct", 0.1))
    max_weight = float(_setting(settings, "max_weight", 0.03))
    mgrs = []
    for fac in factor_weights.columns:
        if fac in factors_df.columns and fac not in mgrs:
            mgrs.append(fac)
    all_symbols = factors_df.index.get_level_values("symbol").unique()
    if len(factor_weights.index) == 0:
        return pd.Series(dtype=float), pd.DataFrame(columns=["long_count", "short_count"])
    factors_df = by_date(factors_df)
    pi = panel_index(factors_df.index)
    dev = device()
    F, D, A = len(mgrs), pi.D, pi.A
    if F:
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
