"""Generate golden input/output vectors by running the REFERENCE implementation.

Test infrastructure only.  Run in the build container (where /root/reference exists):

    python tests/golden/make_golden.py

It imports the reference modules from /root/reference with ``sys.modules`` stubs for the
two third-party packages that are absent from this image and never used on the hot path:

* ``statsmodels.api`` -- dead import at operations.py:3
* ``cvxpy``            -- only used by mvo_selector (factor_selection_methods.py:119-175)
                          and the Simulation MVO solvers (out of scope)

The fixtures are plain data (inputs + reference outputs) written as ``.npz`` (no pickles)
plus ``manifest.json`` recording seeds, shapes and package versions.  Nothing under
/root/reference is copied; the GPU box only ever sees the ``.npz`` files.
"""
from __future__ import annotations

import json
import os
import sys
import types
import warnings

import numpy as np
import pandas as pd

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def import_reference():
    sys.dont_write_bytecode = True
    sm = types.ModuleType("statsmodels")
    sma = types.ModuleType("statsmodels.api")
    sma.OLS = lambda *a, **k: None
    sma.add_constant = lambda *a, **k: None
    sm.api = sma
    cp = types.ModuleType("cvxpy")
    for name in ("Variable", "quad_form", "norm1", "Maximize", "Minimize", "Problem", "sum"):
        setattr(cp, name, lambda *a, **k: None)
    sys.modules.setdefault("statsmodels", sm)
    sys.modules.setdefault("statsmodels.api", sma)
    sys.modules.setdefault("cvxpy", cp)
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import matplotlib
    matplotlib.use("Agg")
    import logging
    logging.disable(logging.CRITICAL)
    import operations as ref_ops  # noqa: E402
    import factor_selector as ref_fs  # noqa: E402
    import factor_selection_methods as ref_fsm  # noqa: E402
    import composite_factor as ref_cf  # noqa: E402
    return ref_ops, ref_fs, ref_fsm, ref_cf


# --------------------------------------------------------------------------- encoding
def enc_index(idx: pd.MultiIndex, dates, syms):
    """(date, symbol) MultiIndex -> two int32 code arrays into ``dates`` / ``syms``."""
    d = pd.Index(dates).get_indexer(idx.get_level_values(0))
    s = pd.Index(syms).get_indexer(idx.get_level_values(1))
    assert (d >= 0).all() and (s >= 0).all()
    return d.astype(np.int32), s.astype(np.int32)


def put_series(store, key, ser: pd.Series, dates, syms):
    d, s = enc_index(ser.index, dates, syms)
    store[key + "__d"] = d
    store[key + "__s"] = s
    store[key + "__v"] = ser.to_numpy(dtype=np.float64, na_value=np.nan)
    store[key + "__name"] = np.array("" if ser.name is None else str(ser.name))
    store[key + "__hasname"] = np.array(ser.name is not None)


# --------------------------------------------------------------------------- panels
def ops_panel(rng, D=60, A=40, ragged=False):
    """Small panel exercising the quirks listed in SURVEY Appendix A."""
    dates = pd.bdate_range("2020-01-01", periods=D)
    syms = [f"S{i:03d}" for i in range(A)]
    x = rng.standard_normal((D, A))
    tie = rng.random((D, A)) < 0.5
    x[tie] = np.round(x[tie], 1)                       # ties
    x[rng.random((D, A)) < 0.10] = np.nan              # 10% NaN
    x[10:41, 3] = 0.3                                  # constant run (ts_std exact zero)
    x[20:26, 5] = 0.1 + 0.2                            # near-constant run
    x[7, :] = np.nan                                   # all-NaN date
    x[30:45, 9] = np.nan                               # long NaN run (ffill)
    x[12, 11] = -0.0                                   # signed zero
    y = 0.5 * np.nan_to_num(x) + rng.standard_normal((D, A))
    y[rng.random((D, A)) < 0.05] = np.nan
    grp = rng.integers(0, 5, size=A).astype(np.float64)  # sector id per symbol (constant)
    G = np.broadcast_to(grp, (D, A)).copy()
    present = np.ones((D, A), dtype=bool)
    if ragged:
        present &= rng.random((D, A)) > 0.15
        present[5, :] = False
        present[5, 17] = True                           # single-asset date
        present[:, 0] = True
    di, si = np.nonzero(present)                        # lexsorted (date, symbol)
    idx = pd.MultiIndex.from_arrays([dates[di], [syms[k] for k in si]], names=["date", "symbol"])
    sx = pd.Series(x[di, si], index=idx, name="fx")
    sy = pd.Series(y[di, si], index=idx, name="fy")
    sg = pd.Series(G[di, si], index=idx, name="grp")
    return dates, syms, sx, sy, sg


def factor_panel(rng, D, A, F, names, dup=True, const=True):
    dates = pd.bdate_range("2019-01-01", periods=D)
    syms = [f"A{i:03d}" for i in range(A)]
    X = rng.standard_normal((D, A, F))
    X[rng.random((D, A, F)) < 0.03] = np.nan
    tie = rng.random((D, A, F)) < 0.05
    X[tie] = np.round(X[tie], 1)
    r = 0.01 * rng.standard_normal((D, A))
    r[1:] += 0.004 * np.nan_to_num(X[:-1, :, 0]) - 0.003 * np.nan_to_num(X[:-1, :, 1])
    r[rng.random((D, A)) < 0.02] = np.nan
    r[4, :] = np.nan                                    # a date with no returns
    r[9, 3:] = np.nan                                   # a date with < 3 valid pairs
    if dup:
        X[:, :, F - 1] = X[:, :, 2]                     # duplicate factor column
    if const:
        X[:, :, F - 2] = 1.25                           # constant factor (pearsonr NaN)
    idx = pd.MultiIndex.from_product([dates, syms], names=["date", "symbol"])
    df = pd.DataFrame(X.reshape(D * A, F), index=idx, columns=names)
    ret = pd.Series(r.reshape(-1), index=idx, name="log_return")
    fret = pd.DataFrame(0.01 * rng.standard_normal((D, F)), index=dates, columns=names)
    fret.index.name = "date"
    return dates, syms, df, ret, fret


# --------------------------------------------------------------------------- generators
def gen_ops(ref_ops, rng, ragged):
    dates, syms, x, y, g = ops_panel(rng, ragged=ragged)
    st = {"dates": np.array([str(d.date()) for d in dates]), "syms": np.array(syms)}
    put_series(st, "in_x", x, dates, syms)
    put_series(st, "in_y", y, dates, syms)
    put_series(st, "in_g", g, dates, syms)
    cases = []

    def add(key, ser):
        put_series(st, "out_" + key, ser, dates, syms)
        cases.append(key)

    for w in (3, 5, 20):
        add(f"ts_sum_{w}", ref_ops.ts_sum(x, w))
        add(f"ts_mean_{w}", ref_ops.ts_mean(x, w))
        add(f"ts_std_{w}", ref_ops.ts_std(x, w))
        add(f"ts_zscore_{w}", ref_ops.ts_zscore(x, w))
        add(f"ts_rank_{w}", ref_ops.ts_rank(x, w))
        add(f"ts_diff_{w}", ref_ops.ts_diff(x, w))
        add(f"ts_delay_{w}", ref_ops.ts_delay(x, w))
        add(f"ts_decay_{w}", ref_ops.ts_decay(x, w))
    add("ts_decay_0", ref_ops.ts_decay(x, 0))
    add("ts_decay_1", ref_ops.ts_decay(x, 1))
    add("ts_backfill", ref_ops.ts_backfill(x))
    for m in ("average", "min", "max", "first", "dense"):
        add(f"cs_rank_{m}", ref_ops.cs_rank(x, method=m))
    add("cs_winsor", ref_ops.cs_winsor(x))
    add("cs_winsor_10_90", ref_ops.cs_winsor(x, limits=(0.1, 0.9)))
    add("cs_filter_center", ref_ops.cs_filter_center(x))
    add("cs_filter_center_20_60", ref_ops.cs_filter_center(x, center=(0.2, 0.6)))
    add("cs_zscore", ref_ops.cs_zscore(x))
    add("cs_mean", ref_ops.cs_mean(x))
    add("cs_bool", ref_ops.cs_bool(x > 0, 1.0, -1.0))
    add("sign", ref_ops.sign(x))
    add("power_2", ref_ops.power(x, 2))
    add("power_0.5", ref_ops.power(x, 0.5))
    add("log", ref_ops.log(x))
    add("abs", ref_ops.abs_(x))
    add("clip", ref_ops.clip(x, -0.5, 0.5))
    add("market_neutralize", ref_ops.market_neutralize(x))
    add("group_mean", ref_ops.group_mean(x, g))
    add("group_neutralize", ref_ops.group_neutralize(x, g))
    add("group_normalize", ref_ops.group_normalize(x, g))
    add("group_rank_normalized", ref_ops.group_rank_normalized(x, g))
    for lag in (0, 1):
        for rt in (0, 1, 2, 3, 6):
            add(f"ts_regression_fast_5_{lag}_{rt}", ref_ops.ts_regression_fast(y, x, 5, lag=lag, rettype=rt))
    for rt in ("resid", "beta", "alpha", "fitted", "r2"):
        add(f"cs_regression_{rt}", ref_ops.cs_regression(y, x, rettype=rt))
    # bucket: categorical labels -> integer codes (-1 = NaN), labels stored separately
    u = ref_ops.cs_rank(x)
    for br in ((0.2, 1.0, 0.2), (0.0, 1.0, 0.25)):
        b = ref_ops.bucket(u, bin_range=br)
        key = "bucket_%g_%g_%g" % br
        d, s = enc_index(b.index, dates, syms)
        st["out_" + key + "__d"], st["out_" + key + "__s"] = d, s
        st["out_" + key + "__codes"] = b.cat.codes.to_numpy().astype(np.int32)
        st["out_" + key + "__labels"] = np.array(list(b.cat.categories))
        put_series(st, "in_" + key, u, dates, syms)
    # DataFrame (column-wise) call path
    dfx = pd.DataFrame({"a": x, "b": y, "c": -x})
    for op, kw in (("ts_mean", {"window": 5}), ("cs_rank", {}), ("cs_zscore", {})):
        out = getattr(ref_ops, op)(dfx, **kw)
        for c in dfx.columns:
            add(f"df_{op}_{c}", out[c])
        put_series(st, f"in_df_{op}_b", dfx["b"], dates, syms)
    return st, cases


def gen_metrics(ref_fs, rng):
    F = 8
    names = [f"g{k // 4:03d}_{k:04d}_{['eq', 'flx', 'long', 'short', 'raw'][k % 5]}" for k in range(F)]
    dates, syms, df, ret, fret = factor_panel(rng, 120, 50, F, names)
    m = ref_fs.single_factor_metrics(df, ret)
    st = {
        "dates": np.array([str(d.date()) for d in dates]), "syms": np.array(syms),
        "names": np.array(names), "X": df.to_numpy().reshape(len(dates), len(syms), F),
        "R": ret.to_numpy().reshape(len(dates), len(syms)),
        "out_order": np.array(list(m.index)), "out_cols": np.array(list(m.columns)),
        "out_vals": m.to_numpy(dtype=np.float64),
    }
    return st


def gen_selector(ref_fs, rng):
    F = 8
    names = [f"g{k // 4:03d}_{k:04d}_{['eq', 'flx', 'long', 'short', 'raw'][k % 5]}" for k in range(F)]
    dates, syms, df, ret, fret = factor_panel(rng, 70, 40, F, names)
    st = {
        "dates": np.array([str(d.date()) for d in dates]), "syms": np.array(syms),
        "names": np.array(names), "X": df.to_numpy().reshape(len(dates), len(syms), F),
        "R": ret.to_numpy().reshape(len(dates), len(syms)), "FR": fret.to_numpy(),
    }
    cases = []
    runs = [
        ("icir_top_w20_top2_thrm1", 20, "icir_top", {"top_x": 2, "icir_threshold": -1}),
        ("icir_top_w20_top5_thr003", 20, "icir_top", {"top_x": 5, "icir_threshold": 0.03}),
        ("icir_top_w20_top3_ic", 20, "icir_top", {"top_x": 3, "icir_threshold": -1, "use_rank_icir": False}),
        ("icir_top_w10_default", 10, "icir_top", {}),
        ("momentum_w20", 20, "momentum", {}),
        ("momentum_w20_cap03", 20, "momentum", {"max_weight": 0.3}),
    ]
    for key, w, meth, kw in runs:
        sel = ref_fs.FactorSelector(df, ret, fret, window=w, method=meth, method_kwargs=kw)
        out = sel.prepare_selection()
        st[f"out_{key}__dates"] = np.array([str(d.date()) for d in out.index])
        st[f"out_{key}__cols"] = np.array(list(out.columns))
        st[f"out_{key}__vals"] = out.to_numpy(dtype=np.float64)
        cases.append({"key": key, "window": w, "method": meth, "kwargs": kw})
    return st, cases


def gen_composite(ref_cf, rng):
    suf = ["eq", "flx", "long", "short", "raw"]
    names = [f"g{k // 3}_{k}_{suf[k % 5]}" for k in range(12)]
    dates, syms, df, ret, fret = factor_panel(rng, 40, 30, 12, names, dup=False, const=False)
    df.iloc[::7, 4] = np.nan
    df.loc[dates[3], names[0]] = np.nan                 # an all-NaN column-date
    df.loc[dates[5], names[1]] = 0.7                    # a constant column-date (high == low)
    st = {"dates": np.array([str(d.date()) for d in dates]), "syms": np.array(syms),
          "names": np.array(names), "X": df.to_numpy().reshape(len(dates), len(syms), 12)}
    cases = []
    sels = {"all": names, "sub": [names[i] for i in (0, 1, 2, 5, 6, 7, 9, 11)]}
    for sk, sel in sels.items():
        for meth in ("zscore", "rank"):
            out = ref_cf.composite_factor_calculation(df, sel, method=meth)
            key = f"cfc_{sk}_{meth}"
            st[f"out_{key}"] = out.to_numpy(dtype=np.float64)
            cases.append(key)
    # selection_df: a subset of dates (and one date absent from the panel), sparse weights
    sel_dates = list(dates[5:35]) + [pd.Timestamp("2030-01-01")]
    W = np.zeros((len(sel_dates), 12))
    for i in range(len(sel_dates)):
        k = rng.choice(12, size=rng.integers(0, 6), replace=False)
        W[i, k] = rng.random(len(k))
    W[3] = 0.0                                          # date with no positive weight
    W[4, [0, 3, 6]] = [0.2, 0.0, 0.8]
    seldf = pd.DataFrame(W, index=pd.DatetimeIndex(sel_dates, name="date"), columns=names)
    seldf = seldf.div(seldf.sum(axis=1), axis=0).fillna(0)
    st["sel_dates"] = np.array([str(d.date()) for d in seldf.index])
    st["sel_W"] = seldf.to_numpy()
    for meth in ("zscore", "rank"):
        out = ref_cf.weighted_composite_factor(df, seldf, method=meth)
        key = f"wcf_{meth}"
        st[f"out_{key}"] = out.to_numpy(dtype=np.float64)
        cases.append(key)
    return st, cases


def gen_ts_corr(rng):
    """Builder-defined ts_corr pinned to pandas (third-party), not to the reference:
    per symbol ``x.rolling(w).corr(y)``."""
    dates, syms, x, y, g = ops_panel(rng)
    st = {"dates": np.array([str(d.date()) for d in dates]), "syms": np.array(syms)}
    put_series(st, "in_x", x, dates, syms)
    put_series(st, "in_y", y, dates, syms)
    for w in (3, 5, 20):
        parts = [xs.rolling(w).corr(y.xs(sym, level="symbol", drop_level=False))
                 for sym, xs in x.groupby(level="symbol")]
        out = pd.concat(parts).reindex(x.index)
        put_series(st, f"out_ts_corr_{w}", out, dates, syms)
    return st


def main():
    warnings.filterwarnings("ignore")
    os.environ["TQDM_DISABLE"] = "1"
    ref_ops, ref_fs, ref_fsm, ref_cf = import_reference()
    import scipy
    manifest = {
        "generator": "tests/golden/make_golden.py",
        "reference": "Yuming-Yang/FactorModeling snapshot 2025-08-24 (/root/reference)",
        "versions": {"numpy": np.__version__, "pandas": pd.__version__, "scipy": scipy.__version__,
                     "python": sys.version.split()[0]},
        "files": {},
    }
    st, cases = gen_ops(ref_ops, np.random.default_rng(100), ragged=False)
    np.savez_compressed(os.path.join(OUT, "ops_dense.npz"), **st)
    manifest["files"]["ops_dense.npz"] = {"seed": 100, "D": 60, "A": 40, "cases": cases}
    st, cases = gen_ops(ref_ops, np.random.default_rng(101), ragged=True)
    np.savez_compressed(os.path.join(OUT, "ops_ragged.npz"), **st)
    manifest["files"]["ops_ragged.npz"] = {"seed": 101, "D": 60, "A": 40, "ragged": True, "cases": cases}
    st = gen_metrics(ref_fs, np.random.default_rng(200))
    np.savez_compressed(os.path.join(OUT, "metrics.npz"), **st)
    manifest["files"]["metrics.npz"] = {"seed": 200, "D": 120, "A": 50, "F": 8}
    st, cases = gen_selector(ref_fs, np.random.default_rng(300))
    np.savez_compressed(os.path.join(OUT, "selector.npz"), **st)
    manifest["files"]["selector.npz"] = {"seed": 300, "D": 70, "A": 40, "F": 8, "cases": cases}
    st, cases = gen_composite(ref_cf, np.random.default_rng(400))
    np.savez_compressed(os.path.join(OUT, "composite.npz"), **st)
    manifest["files"]["composite.npz"] = {"seed": 400, "D": 40, "A": 30, "F": 12, "cases": cases}
    st = gen_ts_corr(np.random.default_rng(500))
    np.savez_compressed(os.path.join(OUT, "ts_corr_pandas.npz"), **st)
    manifest["files"]["ts_corr_pandas.npz"] = {"seed": 500, "D": 60, "A": 40,
                                               "pinned_to": "pandas Rolling.corr (no reference counterpart)"}
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("wrote", sorted(manifest["files"]))


if __name__ == "__main__":
    main()
