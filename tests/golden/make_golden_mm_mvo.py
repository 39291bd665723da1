"""Golden vectors for multi_manager.compute_multimanager_weights with MVO managers
(multi_manager.py:15-29, :32-81; portfolio_simulation.py:96-154 with the scipy SLSQP
'mvo' solver, :183-248), by running the REFERENCE here (test infrastructure only):

    python tests/golden/make_golden_mm_mvo.py      -> tests/golden/mm_mvo.npz

cvxpy is absent from this image: it is stubbed and ``use_cvxpy=False`` runs the scipy
path.  Stored: the inputs, each manager's book (``_daily_trade_list`` output: shifted
weights and counts) and the combined weights / counts.
"""
from __future__ import annotations

import os
import sys
import warnings

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import OUT, import_reference  # noqa: E402


def main():
    warnings.filterwarnings("ignore")
    os.environ["TQDM_DISABLE"] = "1"
    import_reference()
    import multi_manager as mm
    from portfolio_simulation import SimulationSettings
    rng = np.random.default_rng(31)
    D, A, F = 16, 11, 3
    dates = pd.bdate_range("2022-06-01", periods=D)
    syms = [f"M{k:02d}" for k in range(A)]
    idx = pd.MultiIndex.from_product([dates, syms], names=["date", "symbol"])
    X = rng.standard_normal((D * A, F))
    X[rng.random(X.shape) < 0.06] = np.nan
    X[np.arange(D * A) // A == 5, 1] = np.nan          # manager f1 has no rows on date 5
    names = [f"f{k}" for k in range(F)]
    factors_df = pd.DataFrame(X, index=idx, columns=names)
    ret = pd.Series(0.01 * rng.standard_normal(D * A), index=idx, name="ret")
    cap = pd.Series(rng.integers(0, 2, D * A).astype(float), index=idx)
    inv = pd.Series(1.0, index=idx)
    wd = dates[4:]
    fw = pd.DataFrame(rng.random((len(wd), 4)), index=pd.Index(wd, name="date"), columns=["f2", "f0", "zz", "f1"])
    fw.iloc[::4, 1] = 0.0
    fw = fw.div(fw.sum(axis=1), axis=0)
    settings = SimulationSettings(returns=ret, cap_flag=cap, investability_flag=inv, factors_df=factors_df,
                                  method="mvo", use_cvxpy=False, lookback_period=5, plot=False)
    w, counts = mm.compute_multimanager_weights(factors_df, fw, settings)
    st = {"X": X, "D": np.array(D), "A": np.array(A), "R": ret.to_numpy(), "CAP": cap.to_numpy(),
          "fw": fw.to_numpy(), "fw_dates": np.arange(4, D), "fw_cols": np.array(list(fw.columns)),
          "w_d": pd.Index(dates).get_indexer(w.index.get_level_values(0)).astype(np.int32),
          "w_s": pd.Index(syms).get_indexer(w.index.get_level_values(1)).astype(np.int32),
          "w_v": w.to_numpy(dtype=np.float64),
          "counts": counts[["long_count", "short_count"]].to_numpy(dtype=np.float64)}
    for fac in names:
        bw, bc = mm.compute_manager_weights(factors_df[fac].dropna(), settings, name=fac)
        st[f"book_{fac}__d"] = pd.Index(dates).get_indexer(bw.index.get_level_values(0)).astype(np.int32)
        st[f"book_{fac}__s"] = pd.Index(syms).get_indexer(bw.index.get_level_values(1)).astype(np.int32)
        st[f"book_{fac}__v"] = bw.to_numpy(dtype=np.float64)
        st[f"book_{fac}__cd"] = pd.Index(dates).get_indexer(bc.index).astype(np.int32)
        st[f"book_{fac}__c"] = bc[["long_count", "short_count"]].to_numpy(dtype=np.float64)
    np.savez_compressed(os.path.join(OUT, "mm_mvo.npz"), **st)
    print("wrote mm_mvo.npz", len(w), "weights;", counts.shape)


if __name__ == "__main__":
    main()
