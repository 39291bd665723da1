"""Golden vectors for multi_manager.compute_multimanager_weights (multi_manager.py:32-81)
with equal-weight managers, by running the REFERENCE here (test infrastructure only):

    python tests/golden/make_golden_mm.py      -> tests/golden/mm.npz
"""
from __future__ import annotations

import os
import sys

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import OUT, import_reference  # noqa: E402


def main():
    import_reference()
    import multi_manager as mm
    rng = np.random.default_rng(21)
    D, A, F = 22, 37, 4
    dates = pd.bdate_range("2022-03-01", periods=D)
    syms = [f"S{k:03d}" for k in range(A)]
    idx = pd.MultiIndex.from_product([dates, syms], names=["date", "symbol"])
    X = rng.standard_normal((D * A, F))
    X[rng.random(X.shape) < 0.08] = np.nan
    X[np.arange(D * A) // A == 4, 2] = np.nan          # factor 2 absent on date 4
    names = [f"f{k}" for k in range(F)]
    factors_df = pd.DataFrame(X, index=idx, columns=names)
    wd = dates[3:]
    fw = pd.DataFrame(rng.random((len(wd), 4)), index=pd.Index(wd, name="date"),
                      columns=["f2", "f0", "zz", "f3"])
    fw.iloc[::3, 1] = 0.0
    fw = fw.div(fw.sum(axis=1), axis=0)
    settings = dict(returns=None, cap_flag=None, investability_flag=None, factors_df=None,
                    method="equal", pct=0.2, plot=False)
    w, counts = mm.compute_multimanager_weights(factors_df, fw, settings)
    st = {"X": X, "D": np.array(D), "A": np.array(A), "fw": fw.to_numpy(), "fw_dates": np.arange(3, D),
          "fw_cols": np.array(list(fw.columns)), "pct": np.array(0.2),
          "w_d": pd.Index(dates).get_indexer(w.index.get_level_values(0)).astype(np.int32),
          "w_s": pd.Index(syms).get_indexer(w.index.get_level_values(1)).astype(np.int32),
          "w_v": w.to_numpy(dtype=np.float64),
          "counts": counts[["long_count", "short_count"]].to_numpy(dtype=np.float64)}
    np.savez_compressed(os.path.join(OUT, "mm.npz"), **st)
    print("wrote mm.npz", len(w), "weights;", counts.shape)


if __name__ == "__main__":
    main()
