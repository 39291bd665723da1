"""Daily trade list of portfolio_simulation.Simulation on the GPU.

``daily_trade_list(custom_feature, pct)`` returns what ``Simulation._daily_trade_list()``
returns for ``method='equal'`` (portfolio_simulation.py:96-170): the per-symbol
``shift(1)`` of each day's equal-weight long/short book (a Series over the sorted
``(date, symbol)`` rows of ``custom_feature``) and the ``long_count`` / ``short_count``
DataFrame indexed by date.  Computed by ``k_trade_equal`` + the ts delay kernel
(csrc/sim.hip); ``linear`` and the MVO methods stay with the reference (host QP) for now.
"""
from __future__ import annotations

import numpy as np
import pandas as pd
import torch

from . import engine as E
from .panel import device, panel_index


def daily_trade_list(custom_feature: pd.Series, pct: float = 0.1, method: str = "equal"):
    if method != "equal":
        raise NotImplementedError(f"method {method!r}: only 'equal' runs on the device")
    pi = panel_index(custom_feature.index)
    dev = device()
    X = pi.to_device(custom_feature.to_numpy(dtype=np.float64), dev)[0]
    W, counts = E.trade_equal(X, pct, present=pi.present(dev))
    W = W.cpu().numpy().reshape(-1)
    counts = counts.cpu().numpy()
    order = np.sort(pi.flat)
    d, s = order // pi.A, order % pi.A
    index = pd.MultiIndex.from_arrays([pi.dates[d], pi.symbols[s]], names=list(custom_feature.index.names))
    shifted = pd.Series(W[order], index=index)
    counts_df = pd.DataFrame({"long_count": counts[:, 0].astype(np.int64),
                              "short_count": counts[:, 1].astype(np.int64)},
                             index=pd.Index(pi.dates, name=custom_feature.index.names[0]))
    return shifted, counts_df
