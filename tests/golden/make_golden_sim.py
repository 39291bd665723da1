"""Golden vectors for Simulation._daily_trade_list (portfolio_simulation.py:96-170), method
'equal', by running the REFERENCE in this container (test infrastructure only):

    python tests/golden/make_golden_sim.py

Cases: a dense panel (the notebook's ts_decay(...).fillna(0) composite, pipeline.ipynb:268)
and a ragged one (multi_manager.py:44 feeds factors_df[fac].dropna()), plus dates with an
empty leg, continuous values (no exact ties at the k-th value, where numpy's unstable
quicksort order is implementation-defined).  Writes sim.npz (plain arrays, no pickles).
"""
from __future__ import annotations

import os
import sys

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import OUT, import_reference, put_series  # noqa: E402


def case(rng, D, A, ragged):
    dates = pd.bdate_range("2021-01-01", periods=D)
    syms = [f"S{k:04d}" for k in range(A)]
    idx = pd.MultiIndex.from_product([dates, syms], names=["date", "symbol"])
    v = rng.standard_normal(len(idx))
    v[rng.random(len(idx)) < 0.03] = 0.0
    s = pd.Series(v, index=idx)
    grid = v.reshape(D, A)
    grid[3] = np.abs(grid[3]) + 0.1          # no negative leg -> flat day
    grid[5, : A // 2] = np.nan               # NaN values inside a date group
    s = pd.Series(grid.ravel(), index=idx)
    if ragged:
        s = s.dropna()
        drop = rng.random(len(s)) < 0.1
        s = s[~drop]
    return s, dates, syms


def main():
    import_reference()
    import portfolio_simulation as ps
    rng = np.random.default_rng(11)
    st = {}
    for name, D, A, ragged, pct in (("dense", 24, 57, False, 0.1), ("ragged", 30, 83, True, 0.15),
                                    ("small", 6, 7, False, 0.1)):
        s, dates, syms = case(rng, D, A, ragged)
        settings = ps.SimulationSettings(returns=None, cap_flag=None, investability_flag=None,
                                         factors_df=None, method="equal", pct=pct, plot=False)
        sim = ps.Simulation(name="g", custom_feature=s, settings=settings)
        w, counts = sim._daily_trade_list()
        put_series(st, f"{name}_x", s, dates, syms)
        put_series(st, f"{name}_w", w, dates, syms)
        st[f"{name}_counts"] = counts[["long_count", "short_count"]].to_numpy(dtype=np.float64)
        st[f"{name}_count_dates"] = pd.Index(dates).get_indexer(counts.index).astype(np.int32)
        st[f"{name}_dims"] = np.array([D, A], dtype=np.int64)
        st[f"{name}_pct"] = np.array(pct)
    np.savez_compressed(os.path.join(OUT, "sim.npz"), **st)
    print("wrote", os.path.join(OUT, "sim.npz"), {k: v.shape for k, v in st.items() if k.endswith("__v")})


if __name__ == "__main__":
    main()
