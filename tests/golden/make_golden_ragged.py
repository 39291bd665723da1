"""Golden vectors for the ragged / non-contiguous selection paths and the C5 window.

Test infrastructure only.  Run in the build container (where /root/reference exists):

    python tests/golden/make_golden_ragged.py

Imports the reference exactly as make_golden.py does (stubs for the absent, unused
``statsmodels.api`` / ``cvxpy``) and writes plain-data ``.npz`` fixtures:

* ``metrics_ragged.npz`` -- ``single_factor_metrics`` (factor_selector.py:26-73) on a
  ragged panel: rows missing per (date, symbol), a symbol that lists late, a symbol that
  stops early, so ``groupby('symbol').shift(1)`` (:33) lags over each symbol's own rows.
* ``selector_ragged.npz`` -- ``FactorSelector.prepare_selection`` (:94-139) on the same
  kind of panel (icir_top, momentum), and on a dense panel whose ``factor_ret_df`` lacks
  some panel dates (``self.dates`` = intersection, :84-88), which takes the per-window
  general path.
* ``ts_corr60_pandas.npz`` -- the builder-defined ``ts_corr`` (no reference counterpart)
  at the C5 window of 60 rows, pinned to pandas ``Rolling.corr``.
"""
from __future__ import annotations

import json
import os
import sys
import warnings

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import import_reference, put_series  # noqa: E402

NAMES = [f"g{k // 4:03d}_{k:04d}_{['eq', 'flx', 'long', 'short', 'raw'][k % 5]}" for k in range(8)]


def ragged_factor_panel(rng, D, A, F, keep=0.85):
    """Long (date, symbol) frame with missing rows.  Returns the dense [D][A][F] view
    (NaN where a row is absent), the presence mask and the reference-layout inputs."""
    dates = pd.bdate_range("2018-01-01", periods=D)
    syms = [f"Q{i:03d}" for i in range(A)]
    X = rng.standard_normal((D, A, F))
    X[rng.random((D, A, F)) < 0.03] = np.nan
    tie = rng.random((D, A, F)) < 0.05
    X[tie] = np.round(X[tie], 1)
    X[:, :, F - 1] = X[:, :, 2]                          # duplicated factor
    r = 0.01 * rng.standard_normal((D, A))
    r[1:] += 0.004 * np.nan_to_num(X[:-1, :, 0]) - 0.003 * np.nan_to_num(X[:-1, :, 1])
    r[rng.random((D, A)) < 0.02] = np.nan
    present = rng.random((D, A)) < keep
    present[:, 0] = True                                 # one full-history symbol
    present[: D // 3, 1] = False                         # lists late
    present[2 * D // 3:, 2] = False                      # stops early
    present[6, :] = False
    present[6, [4, 9]] = True                            # a date with two rows only
    di, si = np.nonzero(present)                         # lexsorted (date, symbol)
    idx = pd.MultiIndex.from_arrays([dates[di], [syms[k] for k in si]], names=["date", "symbol"])
    df = pd.DataFrame(X[di, si], index=idx, columns=NAMES[:F])
    ret = pd.Series(r[di, si], index=idx, name="log_return")
    fret = pd.DataFrame(0.01 * rng.standard_normal((D, F)), index=dates, columns=NAMES[:F])
    fret.index.name = "date"
    Xd = np.where(present[..., None], X, np.nan)
    Rd = np.where(present, r, np.nan)
    return dates, syms, present, Xd, Rd, df, ret, fret


def base_store(dates, syms, present, Xd, Rd, F):
    return {"dates": np.array([str(d.date()) for d in dates]), "syms": np.array(syms),
            "names": np.array(NAMES[:F]), "present": present, "X": Xd, "R": Rd}


def gen_metrics_ragged(ref_fs, rng):
    dates, syms, present, Xd, Rd, df, ret, fret = ragged_factor_panel(rng, 90, 45, 8)
    m = ref_fs.single_factor_metrics(df, ret)
    st = base_store(dates, syms, present, Xd, Rd, 8)
    st.update(out_order=np.array(list(m.index)), out_vals=m.to_numpy(dtype=np.float64))
    return st


def _run_selector(ref_fs, st, df, ret, fret, runs):
    cases = []
    for key, w, meth, kw in runs:
        out = ref_fs.FactorSelector(df, ret, fret, window=w, method=meth, method_kwargs=kw).prepare_selection()
        st[f"out_{key}__dates"] = np.array([str(d.date()) for d in out.index])
        st[f"out_{key}__cols"] = np.array(list(out.columns))
        st[f"out_{key}__vals"] = out.to_numpy(dtype=np.float64)
        cases.append({"key": key, "window": w, "method": meth, "kwargs": kw})
    return cases


def gen_selector_ragged(ref_fs, rng):
    dates, syms, present, Xd, Rd, df, ret, fret = ragged_factor_panel(rng, 60, 35, 8)
    st = base_store(dates, syms, present, Xd, Rd, 8)
    st["FR"] = fret.to_numpy()
    runs = [("ragged_icir_top_w15_top3", 15, "icir_top", {"top_x": 3, "icir_threshold": -1}),
            ("ragged_momentum_w15", 15, "momentum", {})]
    cases = _run_selector(ref_fs, st, df, ret, fret, runs)
    # dense panel, factor_ret_df missing some panel dates: non-contiguous self.dates
    D, A, F = 55, 30, 8
    dd = pd.bdate_range("2017-03-01", periods=D)
    sy = [f"N{i:03d}" for i in range(A)]
    X = rng.standard_normal((D, A, F))
    X[rng.random((D, A, F)) < 0.03] = np.nan
    r = 0.01 * rng.standard_normal((D, A))
    r[1:] += 0.004 * np.nan_to_num(X[:-1, :, 0])
    idx = pd.MultiIndex.from_product([dd, sy], names=["date", "symbol"])
    df2 = pd.DataFrame(X.reshape(D * A, F), index=idx, columns=NAMES[:F])
    ret2 = pd.Series(r.reshape(-1), index=idx, name="log_return")
    fr_mask = np.ones(D, dtype=bool)
    fr_mask[[5, 17, 18, 40]] = False
    fret2 = pd.DataFrame(0.01 * rng.standard_normal((int(fr_mask.sum()), F)), index=dd[fr_mask], columns=NAMES[:F])
    fret2.index.name = "date"
    st.update(gap_dates=np.array([str(d.date()) for d in dd]), gap_syms=np.array(sy), gap_X=X, gap_R=r,
              gap_fr_mask=fr_mask, gap_FR=fret2.to_numpy())
    runs = [("gap_icir_top_w12_top3", 12, "icir_top", {"top_x": 3, "icir_threshold": -1}),
            ("gap_momentum_w12", 12, "momentum", {})]
    cases += _run_selector(ref_fs, st, df2, ret2, fret2, runs)
    return st, cases


def gen_ts_corr60(rng):
    D, A = 150, 24
    dates = pd.bdate_range("2016-01-01", periods=D)
    syms = [f"C{i:03d}" for i in range(A)]
    x = rng.standard_normal((D, A))
    x[rng.random((D, A)) < 0.02] = np.nan
    x[30:100, 3] = 0.25                                   # constant run: var 0 -> NaN / inf
    y = 0.3 * np.nan_to_num(x) + rng.standard_normal((D, A))
    y[rng.random((D, A)) < 0.02] = np.nan
    present = rng.random((D, A)) < 0.9
    present[:, 0] = True
    di, si = np.nonzero(present)
    idx = pd.MultiIndex.from_arrays([dates[di], [syms[k] for k in si]], names=["date", "symbol"])
    sx = pd.Series(x[di, si], index=idx, name="fx")
    sy = pd.Series(y[di, si], index=idx, name="fy")
    st = {"dates": np.array([str(d.date()) for d in dates]), "syms": np.array(syms)}
    put_series(st, "in_x", sx, dates, syms)
    put_series(st, "in_y", sy, dates, syms)
    parts = [xs.rolling(60).corr(sy.xs(sym, level="symbol", drop_level=False))
             for sym, xs in sx.groupby(level="symbol")]
    put_series(st, "out_ts_corr_60", pd.concat(parts).reindex(sx.index), dates, syms)
    return st


def main():
    warnings.filterwarnings("ignore")
    os.environ["TQDM_DISABLE"] = "1"
    _, ref_fs, _, _ = import_reference()
    path = os.path.join(HERE, "manifest.json")
    manifest = json.load(open(path))
    st = gen_metrics_ragged(ref_fs, np.random.default_rng(600))
    np.savez_compressed(os.path.join(HERE, "metrics_ragged.npz"), **st)
    manifest["files"]["metrics_ragged.npz"] = {"seed": 600, "D": 90, "A": 45, "F": 8, "ragged": True,
                                               "generator": "make_golden_ragged.py"}
    st, cases = gen_selector_ragged(ref_fs, np.random.default_rng(601))
    np.savez_compressed(os.path.join(HERE, "selector_ragged.npz"), **st)
    manifest["files"]["selector_ragged.npz"] = {"seed": 601, "cases": cases, "generator": "make_golden_ragged.py"}
    st = gen_ts_corr60(np.random.default_rng(602))
    np.savez_compressed(os.path.join(HERE, "ts_corr60_pandas.npz"), **st)
    manifest["files"]["ts_corr60_pandas.npz"] = {"seed": 602, "D": 150, "A": 24, "window": 60,
                                                 "pinned_to": "pandas Rolling.corr (no reference counterpart)",
                                                 "generator": "make_golden_ragged.py"}
    with open(path, "w") as f:
        json.dump(manifest, f, indent=1)
    print("wrote metrics_ragged.npz selector_ragged.npz ts_corr60_pandas.npz")


if __name__ == "__main__":
    main()
