"""Drop-in replacement for the reference's ``operations.py`` (operator library).

Same function names, arguments, return types, index order and Series names as
Yuming-Yang/FactorModeling ``operations.py``; the arithmetic runs in the gfx950 kernels
of libfmx (``engine``).  Every operator accepts a ``(date, symbol)``-indexed Series or a
DataFrame of factor columns (processed as one batched ``[F][D][A]`` panel).

Parity: rolling sums/means/stds/zscores/ranks, shifts, cross-sectional ranks, moments,
quantile ops, group ops and regressions reproduce pandas bit-for-bit; ``ts_decay``
(BLAS dot order) and ``log``/``power`` with general exponents agree to <= 1e-12
relative (tests/test_gpu_parity.py).
"""
from __future__ import annotations

import numpy as np
import pandas as pd
import torch

from . import engine
from .panel import device, panel_index
from .profiling import phase

__all__ = [
    "ts_sum", "ts_mean", "ts_std", "ts_zscore", "ts_rank", "ts_diff", "ts_delay", "ts_decay", "ts_backfill",
    "ts_corr", "cs_rank", "cs_winsor", "cs_filter_center", "cs_zscore", "cs_bool", "cs_mean", "sign", "power",
    "log", "abs_", "clip", "bucket", "group_mean", "group_neutralize", "group_normalize",
    "group_rank_normalized", "market_neutralize", "ts_regression_fast", "cs_regression",
]


def _matrix(obj):
    if isinstance(obj, pd.DataFrame):
        return obj.to_numpy(dtype=np.float64, na_value=np.nan)
    return obj.to_numpy(dtype=np.float64, na_value=np.nan)


def _wrap(obj, vals, name=None, keep_name=True):
    if isinstance(obj, pd.DataFrame):
        return pd.DataFrame(vals, index=obj.index, columns=obj.columns)
    return pd.Series(vals[:, 0] if vals.ndim == 2 else vals, index=obj.index,
                     name=(obj.name if keep_name else name))


def _panel_apply(obj, fn, name=None, keep_name=True):
    """Densify ``obj`` onto the device, run ``fn(X, present)`` and gather back."""
    P = panel_index(obj.index)
    dev = device()
    with phase("pandas->dense"):
        xv = _matrix(obj)
    X = P.to_device(xv, dev)
    Y = fn(X, P.present(dev))
    vals = P.from_device(Y)
    with phase("dense->pandas"):
        return _wrap(obj, vals, name, keep_name)


def _ew(obj, op, a=0.0, b=0.0):
    dev = device()
    v = torch.as_tensor(_matrix(obj), device=dev).contiguous()
    out = engine.elementwise(op, v, a, b).cpu().numpy()
    if isinstance(obj, pd.DataFrame):
        return pd.DataFrame(out, index=obj.index, columns=obj.columns)
    return pd.Series(out, index=obj.index, name=obj.name)


# ========== Time-Series Operations (operations.py:5-51) ==========
def ts_sum(series, window: int):
    """operations.py:6-7"""
    return _panel_apply(series, lambda X, p: engine.ts("sum", X, window, p))


def ts_mean(series, window: int):
    """operations.py:10-11"""
    return _panel_apply(series, lambda X, p: engine.ts("mean", X, window, p))


def ts_std(series, window: int):
    """operations.py:14-15"""
    return _panel_apply(series, lambda X, p: engine.ts("std", X, window, p))


def ts_zscore(series, window: int):
    """operations.py:18-21"""
    return _panel_apply(series, lambda X, p: engine.ts("zscore", X, window, p))


def ts_rank(series, window: int):
    """operations.py:23-32"""
    return _panel_apply(series, lambda X, p: engine.ts("rank", X, window, p))


def ts_diff(series, window: int):
    """operations.py:34-35"""
    return _panel_apply(series, lambda X, p: engine.ts("diff", X, window, p))


def ts_delay(series, window: int):
    """operations.py:37-38"""
    return _panel_apply(series, lambda X, p: engine.ts("delay", X, window, p))


def ts_decay(series, window: int):
    """operations.py:40-48 (window < 1 returns the input object itself)."""
    if window < 1:
        return series
    return _panel_apply(series, lambda X, p: engine.ts("decay", X, window, p))


def ts_backfill(series):
    """operations.py:50-51"""
    return _panel_apply(series, lambda X, p: engine.ts("backfill", X, 1, p))


def ts_corr(x, y, window: int):
    """Builder-defined (no reference counterpart): per-symbol ``x.rolling(window).corr(y)``
    with pandas semantics; ``y`` is aligned to ``x``'s index.  Series or DataFrame ``x``."""
    yv = y.reindex(x.index).to_numpy(dtype=np.float64, na_value=np.nan)
    P = panel_index(x.index)
    dev = device()
    Yd = P.to_device(yv, dev)[0]

    return _panel_apply(x, lambda X, p: engine.ts_corr(X, Yd, window, p))


# ========== Cross section (operations.py:53-86) ==========
def cs_rank(series, method="average"):
    """operations.py:54-62"""
    return _panel_apply(series, lambda X, p: engine.cs_rank(X, method, p))


def _pandas_q(q):
    # pandas Series.quantile hands q*100 to np.percentile, which divides by 100 again
    return float(np.true_divide(np.asarray([q], dtype=np.float64) * 100.0, 100)[0])


def cs_winsor(series, limits=(0.01, 0.99)):
    """operations.py:64-68"""
    qlo, qhi = _pandas_q(limits[0]), _pandas_q(limits[1])
    return _panel_apply(series, lambda X, p: engine.cs_quantile_op("winsor", X, qlo, qhi, p))


def cs_filter_center(series, center=(0.3, 0.7)):
    """operations.py:70-75"""
    qlo, qhi = _pandas_q(center[0]), _pandas_q(center[1])
    return _panel_apply(series, lambda X, p: engine.cs_quantile_op("filter_center", X, qlo, qhi, p))


def cs_zscore(series):
    """operations.py:77-78"""
    return _panel_apply(series, lambda X, p: engine.cs_moment("zscore", X, p))


def cs_bool(condition, true_value: float, false_value: float):
    """operations.py:80-84 -- unnamed Series on condition.index."""
    dev = device()
    c = torch.as_tensor(np.asarray(condition, dtype=bool).astype(np.float64), device=dev)
    out = engine.elementwise("where", c, true_value, false_value).cpu().numpy()
    return pd.Series(out, index=condition.index)


def cs_mean(series):
    """operations.py:85-86"""
    return _panel_apply(series, lambda X, p: engine.cs_moment("mean", X, p))


# ========== Math (operations.py:88-101) ==========
def sign(series):
    return _ew(series, "sign")


def power(series, exp: float):
    return _ew(series, "power", float(exp))


def log(series):
    return _ew(series, "log")


def abs_(series):
    return _ew(series, "abs")


def clip(series, lower, upper):
    return _ew(series, "clip", float(lower), float(upper))


# ========== Group Operations (operations.py:103-168) ==========
def bucket(series, bin_range=(0.2, 1.0, 0.2)):
    """operations.py:104-110 -- categorical labels group1..groupK (pd.cut, right-closed,
    include_lowest); rows come out in date-group order like groupby(...).apply."""
    low, up, step = bin_range
    edges = np.arange(low, up + 1e-8, step)
    labels = [f"group{i + 1}" for i in range(len(edges) - 1)]
    dev = device()
    v = torch.as_tensor(series.to_numpy(dtype=np.float64, na_value=np.nan), device=dev)
    codes = engine.bucket_codes(v, edges).cpu().numpy()
    P = panel_index(series.index)
    order = np.argsort(P.d, kind="stable")
    cat = pd.Categorical.from_codes(codes[order], categories=labels, ordered=True)
    return pd.Series(cat, index=series.index[order], name=series.name)


def _group_ids(series, group):
    g = group.reindex(series.index) if not group.index.equals(series.index) else group
    codes, uniq = pd.factorize(g, sort=True)
    return codes.astype(np.int32), len(uniq)


def _group_apply(series, group, op, method="average"):
    P = panel_index(series.index)
    dev = device()
    codes, ng = _group_ids(series, group)
    Gd = np.full(P.D * P.A, -1, dtype=np.int32)
    Gd[P.flat] = codes
    G = torch.as_tensor(Gd.reshape(P.D, P.A), device=dev)
    X = P.to_device(_matrix(series), dev)
    Y = engine.group_op(op, X, G, ng, method, P.present(dev))
    return pd.Series(P.from_device(Y)[:, 0], index=series.index, name="val")


def group_mean(series, group):
    """operations.py:112-122"""
    return _group_apply(series, group, "mean")


def group_neutralize(series, group):
    """operations.py:124-134"""
    return _group_apply(series, group, "neutralize")


def group_normalize(series, group):
    """operations.py:137-149"""
    return _group_apply(series, group, "normalize")


def group_rank_normalized(series, group, method="average"):
    """operations.py:152-168"""
    return _group_apply(series, group, "rank", method)


def market_neutralize(series):
    """operations.py:171-182"""
    return _panel_apply(series, lambda X, p: engine.cs_moment("market_neutralize", X, p))


# ========== Regressions (operations.py:185-304) ==========
def ts_regression_fast(y, x, window: int, lag: int = 0, rettype: int = 2):
    """operations.py:185-246 -- rolling per-symbol OLS via moments.  ``x.shift(lag)`` is
    the reference's global row shift; rows with NaN y or shifted x are dropped; the
    result keeps non-NaN rows only, sorted by (date, symbol)."""
    if rettype not in (0, 1, 2, 3, 6):
        raise ValueError("rettype not implemented")
    xs = x.shift(lag)
    df = pd.DataFrame({"y": y, "x": xs})
    P = panel_index(df.index)
    dev = device()
    yv = df["y"].to_numpy(dtype=np.float64, na_value=np.nan)
    xv = df["x"].to_numpy(dtype=np.float64, na_value=np.nan)
    ok = ~np.isnan(yv) & ~np.isnan(xv)
    Yd = P.to_device(yv, dev)[0]
    Xd = P.to_device(xv, dev)[0]
    valid = np.zeros(P.D * P.A, dtype=np.uint8)
    valid[P.flat[ok]] = 1
    Vd = torch.as_tensor(valid.reshape(P.D, P.A), device=dev)
    out = engine.ts_regression(Yd, Xd, Vd, window, rettype).cpu().numpy().reshape(-1)
    cells = P.flat[ok]
    vals = out[cells]
    keep = ~np.isnan(vals)
    cells, vals = cells[keep], vals[keep]
    order = np.argsort(cells, kind="stable")           # (date, symbol) lexicographic
    cells, vals = cells[order], vals[order]
    idx = pd.MultiIndex.from_arrays([P.dates[cells // P.A], P.symbols[cells % P.A]], names=["date", "symbol"])
    return pd.Series(vals, index=idx)


def cs_regression(y, x, rettype: str = "resid"):
    """operations.py:248-304 -- per-date OLS, reindexed onto y.index."""
    if rettype not in ("resid", "beta", "alpha", "fitted", "r2"):
        raise ValueError(f"ERROR: rettype={rettype}")
    P = panel_index(y.index)
    dev = device()
    xv = x.reindex(y.index).to_numpy(dtype=np.float64, na_value=np.nan)
    Yd = P.to_device(y.to_numpy(dtype=np.float64, na_value=np.nan), dev)[0]
    Xd = P.to_device(xv, dev)[0]
    out = engine.cs_regression(Yd, Xd, rettype, P.present(dev))
    return pd.Series(P.from_device(out[None])[:, 0], index=y.index)
