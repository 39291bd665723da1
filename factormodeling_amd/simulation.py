"""Daily trade list of portfolio_simulation.Simulation on the GPU.

``daily_trade_list(custom_feature, pct)`` returns what ``Simulation._daily_trade_list()``
returns for ``method='equal'`` (portfolio_simulation.py:96-170): the per-symbol
``shift(1)`` of each day's equal-weight long/short book (a Series over the sorted
``(date, symbol)`` rows of ``custom_feature``) and the ``long_count`` / ``short_count``
DataFrame indexed by date.  Computed by ``k_trade_equal`` / ``k_trade_linear`` (normalised
legs + cap-and-redistribute, :172-181, :250-313) and the per-symbol shift (csrc/sim.hip);
the MVO methods are host QPs (cvxpy) and stay with the reference.
"""
from __future__ import annotations

import numpy as np
import pandas as pd
import torch

from . import engine as E
from .panel import device, panel_index


def by_date(obj):
    """Rows stably reordered by date when they are not: the trade list groups by date and
    shifts per symbol after sort_index() (portfolio_simulation.py:99, :150-151), so the
    row order across dates does not matter -- but the order inside a date does (linear
    weights' pairwise sums), and a stable sort keeps it."""
    dl = obj.index.get_level_values(0)
    if dl.is_monotonic_increasing:
        return obj
    return obj.iloc[np.argsort(dl.values, kind="stable")]


def trade_books(pi, values: np.ndarray, method: str, pct: float, max_weight: float, nan_absent: bool):
    """Trade books of the F signal columns ``values`` [n][F] over ``pi``'s rows: (shifted
    books [F][D][A], counts [F][D][2]) on the device.  The 'linear' weights are numpy
    pairwise sums over each date's rows in INPUT order (groupby('date') keeps it), so when
    that order is not the sorted-symbol order the kernel runs on a per-date row layout
    and the same-day books are scattered back to symbol columns before the shift."""
    dev = device()
    v = np.asarray(values, dtype=np.float64)
    if v.ndim == 1:
        v = v[:, None]
    pos, width, sorted_within = pi.row_layout()
    if method == "equal" or sorted_within:
        X = torch.as_tensor(pi.to_dense(v), device=dev)
        return E.trade_books(X, method, pct, max_weight, present=pi.present(dev), nan_absent=nan_absent)
    F = v.shape[1]
    Xr = np.full((F, pi.D, width), np.nan)
    Xr[:, pi.d, pos] = v.T
    pr = np.zeros((pi.D, width), dtype=np.uint8)
    pr[pi.d, pos] = 1
    _, counts, Wr = E.trade_books(torch.as_tensor(Xr, device=dev), method, pct, max_weight,
                                  present=torch.as_tensor(pr, device=dev), nan_absent=nan_absent, raw=True)
    d_t = torch.as_tensor(pi.d, device=dev)
    W = torch.full((F, pi.D, pi.A), float("nan"), dtype=torch.float64, device=dev)
    W[:, d_t, torch.as_tensor(pi.s, device=dev)] = Wr[:, d_t, torch.as_tensor(pos, device=dev)]
    return E.shift_rows(W), counts


def daily_trade_list(custom_feature: pd.Series, pct: float = 0.1, method: str = "equal", max_weight: float = 0.03):
    if method not in ("equal", "linear"):
        raise NotImplementedError(f"method {method!r}: the device runs 'equal' and 'linear' (MVO is a host QP)")
    custom_feature = by_date(custom_feature)
    pi = panel_index(custom_feature.index)
    W, counts = trade_books(pi, custom_feature.to_numpy(dtype=np.float64), method, pct, max_weight, False)
    W = W[0].cpu().numpy().reshape(-1)
    counts = counts[0].cpu().numpy()
    order = np.sort(pi.flat)
    d, s = order // pi.A, order % pi.A
    index = pd.MultiIndex.from_arrays([pi.dates[d], pi.symbols[s]], names=list(custom_feature.index.names))
    shifted = pd.Series(W[order], index=index)
    counts_df = pd.DataFrame({"long_count": counts[:, 0].astype(np.int64),
                              "short_count": counts[:, 1].astype(np.int64)},
                             index=pd.Index(pi.dates, name=custom_feature.index.names[0]))
    return shifted, counts_df
