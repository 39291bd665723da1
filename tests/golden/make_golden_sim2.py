"""Golden vectors for the rest of portfolio_simulation's per-date path, by running the
REFERENCE in this container (test infrastructure only):

    python tests/golden/make_golden_sim2.py      -> tests/golden/sim2.npz

* ``Simulation._daily_trade_list`` with method 'linear' (portfolio_simulation.py:172-181,
  _normalize_legs :250-262, _cap_and_redistribute :264-313): a dense panel where the cap
  binds, a ragged one, a tiny universe where the redistribution runs out of room, and a
  flat day;
* ``_daily_portfolio_returns`` (:748-797) and ``_calculate_metrics`` (:799-819) on equal
  and linear books with returns / cap flags that cover extra dates and symbols, with and
  without transaction cost, with contributors;
* ``multi_manager.compute_multimanager_weights`` (multi_manager.py:32-81) with linear
  managers on a universe where a symbol that sorts first lists late (symbol order).
Plain arrays only (no pickles).
"""
from __future__ import annotations

import os
import sys
import warnings

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import OUT, import_reference, put_series  # noqa: E402


def signal(rng, D, A, ragged, prefix="S"):
    dates = pd.bdate_range("2021-01-01", periods=D)
    syms = [f"{prefix}{k:04d}" for k in range(A)]
    idx = pd.MultiIndex.from_product([dates, syms], names=["date", "symbol"])
    grid = rng.standard_normal((D, A))
    grid[rng.random((D, A)) < 0.03] = 0.0
    grid[2] = np.abs(grid[2]) + 0.1          # no negative leg -> flat day
    grid[4, : A // 2] = np.nan               # NaN values inside a date group
    grid[6, :3] = [5.0, 4.0, 3.0]            # a few dominant longs: the cap binds hard
    s = pd.Series(grid.ravel(), index=idx)
    if ragged:
        s = s.dropna()
        s = s[~(rng.random(len(s)) < 0.1)]
    return s, dates, syms


def market(rng, dates, syms, extra_dates=2, extra_syms=3):
    """returns / cap_flag over MORE dates and symbols than the signal (alignment cases)."""
    dd = pd.bdate_range(dates[0], periods=len(dates) + extra_dates)
    ss = list(syms) + [f"X{k:02d}" for k in range(extra_syms)]
    idx = pd.MultiIndex.from_product([dd, ss], names=["date", "symbol"])
    r = 0.01 * rng.standard_normal(len(idx))
    r[rng.random(len(idx)) < 0.03] = np.nan
    cap = rng.integers(1, 4, len(idx)).astype(np.float64)
    cap[rng.random(len(idx)) < 0.05] = np.nan
    cap[rng.random(len(idx)) < 0.02] = 4.0      # an unmapped code (kept as the number)
    return pd.Series(r, index=idx), pd.Series(cap, index=idx), dd, ss


def put_frame_result(st, key, res, dates):
    st[f"{key}_res_d"] = pd.Index(dates).get_indexer(pd.DatetimeIndex(res["date"])).astype(np.int32)
    st[f"{key}_res_v"] = res[["log_return", "long_return", "short_return", "long_turnover", "short_turnover",
                              "turnover"]].to_numpy(dtype=np.float64)


def main():
    warnings.filterwarnings("ignore")
    import_reference()
    import multi_manager as mm
    import portfolio_simulation as ps
    rng = np.random.default_rng(77)
    st = {}
    cases = [("lin_dense", 20, 57, False, "linear", 0.03), ("lin_ragged", 24, 83, True, "linear", 0.025),
             ("lin_tiny", 8, 7, False, "linear", 0.2), ("lin_nocap", 10, 40, False, "linear", 1.0),
             ("eq_pnl", 16, 45, True, "equal", 0.03)]
    for name, D, A, ragged, method, mw in cases:
        s, dates, syms = signal(rng, D, A, ragged)
        ret, cap, dd, ss = market(rng, dates, syms)
        inv = pd.Series(1.0, index=ret.index)
        for tc in (True, False):
            settings = ps.SimulationSettings(returns=ret, cap_flag=cap, investability_flag=inv, factors_df=None,
                                             method=method, pct=0.15, max_weight=mw, plot=False,
                                             transaction_cost=tc, contributor=True)
            sim = ps.Simulation(name="g", custom_feature=s, settings=settings)
            w, counts = sim._daily_trade_list()
            res, tl, tsh = sim._daily_portfolio_returns(w)
            key = f"{name}_tc{int(tc)}"
            put_frame_result(st, key, res, dd)
            st[f"{key}_top_long_s"] = np.array(list(tl.index))
            st[f"{key}_top_long_v"] = tl.to_numpy(dtype=np.float64)
            st[f"{key}_top_short_s"] = np.array(list(tsh.index))
            st[f"{key}_top_short_v"] = tsh.to_numpy(dtype=np.float64)
            if tc:
                put_series(st, f"{name}_x", s, dd, ss)
                put_series(st, f"{name}_w", w, dd, ss)
                st[f"{name}_counts"] = counts[["long_count", "short_count"]].to_numpy(dtype=np.float64)
                st[f"{name}_count_dates"] = pd.Index(dd).get_indexer(counts.index).astype(np.int32)
                put_series(st, f"{name}_ret", ret, dd, ss)
                put_series(st, f"{name}_cap", cap, dd, ss)
                st[f"{name}_dims"] = np.array([D, A, len(dd), len(ss)], dtype=np.int64)
                st[f"{name}_mw"] = np.array(mw)
                st[f"{name}_method"] = np.array(method)
                # _calculate_metrics on the same book (alpha = the signal times investability)
                sim.custom_feature = sim.custom_feature * inv
                m = sim._calculate_metrics(w, counts)
                st[f"{name}_metrics"] = m.to_numpy(dtype=np.float64).ravel()
                st[f"{name}_metric_cols"] = np.array(list(m.columns))
    # multi-manager, linear managers, a late-listing symbol that sorts first
    D, A, F = 18, 29, 3
    dates = pd.bdate_range("2022-03-01", periods=D)
    syms = [f"M{k:03d}" for k in range(A)]
    rows = [(d, s_) for d in dates for s_ in syms] + [(d, "A000") for d in dates[7:]]
    idx = pd.MultiIndex.from_tuples(rows, names=["date", "symbol"])
    X = rng.standard_normal((len(idx), F))
    X[rng.random(X.shape) < 0.08] = np.nan
    names = [f"f{k}" for k in range(F)]
    factors_df = pd.DataFrame(X, index=idx, columns=names).sort_index(level="date", sort_remaining=False)
    fw = pd.DataFrame(rng.random((D - 2, 3)), index=pd.Index(dates[2:], name="date"), columns=["f2", "f0", "f1"])
    fw.iloc[::4, 0] = 0.0
    fw = fw.div(fw.sum(axis=1), axis=0)
    settings = dict(returns=None, cap_flag=None, investability_flag=None, factors_df=None, method="linear",
                    pct=0.2, max_weight=0.08, plot=False)
    w, counts = mm.compute_multimanager_weights(factors_df, fw, settings)
    st["mm_dates"] = np.array([str(d.date()) for d in dates])
    st["mm_index_date"] = pd.Index(dates).get_indexer(factors_df.index.get_level_values(0)).astype(np.int32)
    st["mm_index_sym"] = np.array(list(factors_df.index.get_level_values(1)))
    st["mm_X"] = factors_df.to_numpy()
    st["mm_fw"] = fw.to_numpy()
    st["mm_fw_cols"] = np.array(list(fw.columns))
    st["mm_w_d"] = pd.Index(dates).get_indexer(w.index.get_level_values(0)).astype(np.int32)
    st["mm_w_s"] = np.array(list(w.index.get_level_values(1)))
    st["mm_w_v"] = w.to_numpy(dtype=np.float64)
    st["mm_counts"] = counts[["long_count", "short_count"]].to_numpy(dtype=np.float64)
    np.savez_compressed(os.path.join(OUT, "sim2.npz"), **st)
    print("wrote sim2.npz:", len(st), "arrays")


if __name__ == "__main__":
    main()
