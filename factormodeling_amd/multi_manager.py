"""multi_manager.compute_multimanager_weights on the GPU.

Reference: multi_manager.py:32-81.  Each factor is a manager whose book is
Simulation._daily_trade_list over ``factors_df[fac].dropna()`` (method 'equal' only here:
``k_trade_equal`` per factor), and each weight date folds the managers' books and counts
in ``factor_weights`` column order (``k_mm_combine``).  Returns the reference's
``(final_weights, final_counts)``: nonzero weights over ``(date, symbol)`` with symbols in
first-appearance order, counts indexed by date.
"""
from __future__ import annotations

import numpy as np
import pandas as pd
import torch

from . import engine as E
from .panel import device, panel_index


def _setting(settings, key, default):
    if isinstance(settings, dict):
        return settings.get(key, default)
    return getattr(settings, key, default)


def compute_multimanager_weights(factors_df: pd.DataFrame, factor_weights: pd.DataFrame, settings):
    method = _setting(settings, "method", "equal")
    if method != "equal":
        raise NotImplementedError(f"method {method!r}: only 'equal' managers run on the device")
    pct = float(_setting(settings, "pct", 0.1))
    mgrs = []
    for fac in factor_weights.columns:
        if fac in factors_df.columns and fac not in mgrs:
            mgrs.append(fac)
    all_symbols = factors_df.index.get_level_values("symbol").unique()
    if len(factor_weights.index) == 0:
        return pd.Series(dtype=float), pd.DataFrame(columns=["long_count", "short_count"])
    pi = panel_index(factors_df.index)
    dev = device()
    F, D, A = len(mgrs), pi.D, pi.A
    Wf = torch.empty((max(F, 1), D, A), dtype=torch.float64, device=dev)
    cnt = torch.full((max(F, 1), D, 2), float("nan"), dtype=torch.float64, device=dev)
    if F:
        X = pi.to_dense(factors_df[mgrs].to_numpy(dtype=np.float64))
        base = np.ones((D, A), dtype=bool) if pi.present_np is None else pi.present_np.astype(bool)
        for f in range(F):
            pres = torch.as_tensor((base & ~np.isnan(X[f])).astype(np.uint8), device=dev)
            W, c = E.trade_equal(torch.as_tensor(X[f], device=dev), pct, present=pres)
            Wf[f] = W
            cnt[f] = c
    colmap = [mgrs.index(c) if c in mgrs else -1 for c in factor_weights.columns]
    wdate = pi.dates.get_indexer(factor_weights.index)
    out, oc = E.mm_combine(Wf, cnt, factor_weights.to_numpy(dtype=np.float64), colmap, wdate)
    perm = pi.symbols.get_indexer(all_symbols)
    out = out.cpu().numpy()[:, perm]
    oc = oc.cpu().numpy()
    index = pd.MultiIndex.from_product([factor_weights.index, all_symbols], names=["date", "symbol"])
    final = pd.Series(out.reshape(-1), index=index)
    final = final[final != 0]
    counts = pd.DataFrame({"long_count": oc[:, 0], "short_count": oc[:, 1]},
                          index=pd.Index(factor_weights.index, name="date"))
    return final, counts
