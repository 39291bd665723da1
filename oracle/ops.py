"""Oracle restatement of operations.py on the dense panel layout.

Test infrastructure only (see oracle/__init__.py).

Layout: ``x`` is ``float64[D][A]`` (dates x assets).  ``present`` is an optional
``bool[D][A]``: ``False`` marks a (date, symbol) pair that has no row in the
reference's long MultiIndex.  Time-series operators walk each symbol's *present*
rows in date order (the reference is row-based: ``groupby(level='symbol')`` +
``rolling``/``shift``); cross-sectional operators reduce over the present rows of
one date.  Outputs are ``NaN`` where not present.
"""
from __future__ import annotations

import numpy as np

from . import numerics as nm


# --------------------------------------------------------------------------- helpers
def _compact(x, present):
    """Per column, move present rows to the top (date order).  Returns (xc, rows)
    where ``rows[k, a]`` is the source date of compacted row k (or -1)."""
    D, A = x.shape
    if present is None:
        return x.copy(), None
    order = np.argsort(~present, axis=0, kind="stable")          # present first, date order
    cnt = present.sum(axis=0)
    xc = np.take_along_axis(x, order, axis=0)
    k = np.arange(D)[:, None]
    valid = k < cnt[None, :]
    xc = np.where(valid, xc, np.nan)
    rows = np.where(valid, order, -1)
    return xc, rows


def _expand(yc, rows, shape):
    if rows is None:
        return yc
    out = np.full(shape, np.nan)
    k, a = np.nonzero(rows >= 0)
    out[rows[k, a], a] = yc[k, a]
    return out


def _ts(x, present, fn):
    xc, rows = _compact(np.asarray(x, dtype=np.float64), present)
    return _expand(fn(xc), rows, x.shape)


def _mask_out(out, present):
    if present is not None:
        out = np.where(present, out, np.nan)
    return out


# --------------------------------------------------------------------------- time series
def ts_sum(x, window, present=None):
    """operations.py:6-7 -- rolling(window).sum() per symbol."""
    return _ts(x, present, lambda c: nm.roll_sum(c, window))


def ts_mean(x, window, present=None):
    """operations.py:10-11 -- rolling(window).mean() per symbol."""
    return _ts(x, present, lambda c: nm.roll_mean(c, window))


def ts_std(x, window, present=None):
    """operations.py:14-15 -- rolling(window).std() (ddof=1, zsqrt)."""
    return _ts(x, present, lambda c: nm.zsqrt(nm.roll_var(c, window, 1)))


def ts_zscore(x, window, present=None):
    """operations.py:18-21 -- (x - mean) / std.replace(0, nan)."""
    def f(c):
        m = nm.roll_mean(c, window)
        s = nm.zsqrt(nm.roll_var(c, window, 1))
        s = np.where(s == 0, np.nan, s)
        with np.errstate(all="ignore"):
            return (c - m) / s
    return _ts(x, present, f)


def ts_rank(x, window, present=None):
    """operations.py:23-32 -- pct rank (average ties) of the last element of each full
    window: (#less + (#equal + 1) / 2) / window; NaN anywhere in the window -> NaN."""
    def f(c):
        T = c.shape[0]
        out = np.full(c.shape, np.nan)
        for i in range(window - 1, T):
            win = c[i - window + 1:i + 1]
            last = win[-1]
            ok = ~np.isnan(win).any(axis=0)
            less = (win < last).sum(axis=0)
            eq = (win == last).sum(axis=0)
            r = (less + (eq + 1) / 2.0) / window
            out[i] = np.where(ok, r, np.nan)
        return out
    if window < 1:
        raise ValueError("window must be >= 1")
    return _ts(x, present, f)


def _shift_rows(c, k):
    out = np.full(c.shape, np.nan)
    if k > 0:
        out[k:] = c[:-k]
    elif k < 0:
        out[:k] = c[-k:]
    else:
        out[:] = c
    return out


def ts_diff(x, window, present=None):
    """operations.py:34-35 -- x.diff(window) per symbol (row-based)."""
    if present is not None and window < 0:
        # a negative row shift looks ahead within each symbol's compacted rows
        pass
    return _ts(x, present, lambda c: c - _shift_rows(c, window))


def ts_delay(x, window, present=None):
    """operations.py:37-38 -- x.shift(window) per symbol (row-based)."""
    return _ts(x, present, lambda c: _shift_rows(c, window))


def ts_decay(x, window, present=None):
    """operations.py:40-48 -- linearly weighted moving average, weights 1..window
    (newest heaviest), min_periods=window; window < 1 returns the input."""
    x = np.asarray(x, dtype=np.float64)
    if window < 1:
        return x.copy() if present is None else _mask_out(x.copy(), present)
    wts = np.arange(1, window + 1, dtype=np.float64)
    den = float(np.arange(1, window + 1).sum())

    def f(c):
        T = c.shape[0]
        out = np.full(c.shape, np.nan)
        for i in range(window - 1, T):
            win = c[i - window + 1:i + 1]
            ok = ~np.isnan(win).any(axis=0)
            out[i] = np.where(ok, np.tensordot(wts, np.where(ok, win, 0.0), axes=(0, 0)) / den, np.nan)
        return out
    return _ts(x, present, f)


def ts_backfill(x, present=None):
    """operations.py:50-51 -- per-symbol forward fill (unbounded)."""
    def f(c):
        out = c.copy()
        for i in range(1, c.shape[0]):
            out[i] = np.where(np.isnan(out[i]), out[i - 1], out[i])
        return out
    return _ts(x, present, f)


def ts_corr(x, y, window, present=None):
    """Builder-defined (no reference counterpart; pinned to pandas, not the reference):
    per-symbol ``x.rolling(window).corr(y)``.  pandas ``Rolling.corr`` = prep_binary NaN
    propagation, then (mean(xy) - mean(x) mean(y)) * (c / (c - 1)) / sqrt(var(x) var(y))
    with roll_mean / roll_sum(notna, minp=0) / roll_var (ddof=1)."""
    def f(cx, cy):
        with np.errstate(all="ignore"):
            xv = cx + 0 * cy
            yv = cy + 0 * cx
            mxy = nm.roll_mean(xv * yv, window)
            mx = nm.roll_mean(xv, window)
            my = nm.roll_mean(yv, window)
            # roll_sum with min_periods=0: windows are never NaN
            cnt = _roll_count(~np.isnan(xv + yv), window)
            vx = nm.roll_var(xv, window, 1)
            vy = nm.roll_var(yv, window, 1)
            num = (mxy - mx * my) * (cnt / (cnt - 1))
            den = (vx * vy) ** 0.5
            return num / den
    xc, rows = _compact(np.asarray(x, dtype=np.float64), present)
    yc, _ = _compact(np.asarray(y, dtype=np.float64), present)
    return _expand(f(xc, yc), rows, x.shape)


def corr_vol_feature(x, y, window):
    """C5's feature (builder-defined; no reference counterpart): the 60-day
    ts_corr / ts_std of BASELINE configs[4] feeding the composite as
    ``sign(ts_corr(x, y, w)) * (x / ts_std(x, w).replace(0, NaN))`` -- each factor
    sign-aligned with its own recent return correlation and scaled by its own rolling
    volatility (ts_std = operations.py:14-15, the replace(0, NaN) guard of ts_zscore
    :18-21).  np.sign: +-0 -> +0, NaN -> NaN."""
    s = ts_std(x, window)
    c = ts_corr(x, y, window)
    with np.errstate(all="ignore"):
        return np.sign(c) * (x / np.where(s == 0, np.nan, s))


def _roll_count(ok, window):
    c = np.cumsum(ok.astype(np.int64), axis=0)
    out = c.copy()
    out[window:] = c[window:] - c[:-window]
    return out.astype(np.float64)


# --------------------------------------------------------------------------- cross section
def _row_iter(x, present):
    D, A = x.shape
    for d in range(D):
        idx = np.arange(A) if present is None else np.nonzero(present[d])[0]
        yield d, idx


def cs_rank(x, present=None, method="average"):
    """operations.py:54-62 -- rank(method) then (r-1)/(len-1), len counting NaN rows;
    a single-row date gives 0.5."""
    out = np.full(x.shape, np.nan)
    for d, idx in _row_iter(x, present):
        n = len(idx)
        if n == 0:
            continue
        if n == 1:
            out[d, idx] = 0.5
            continue
        r = nm.series_rank(x[d, idx], method)
        out[d, idx] = (r - 1) / (n - 1)
    return out


def cs_winsor(x, present=None, limits=(0.01, 0.99)):
    """operations.py:64-68 -- clip to Series.quantile(limits) when >= 5 non-NaN."""
    qlo, qhi = nm.pandas_quantile_q(limits[0]), nm.pandas_quantile_q(limits[1])
    out = np.full(x.shape, np.nan)
    for d, idx in _row_iter(x, present):
        v = x[d, idx]
        clean = np.sort(v[~np.isnan(v)])
        if len(clean) >= 5:
            lo = nm.percentile_linear(clean, qlo)
            hi = nm.percentile_linear(clean, qhi)
            v = np.where(v < lo, lo, np.where(v > hi, hi, v))
        out[d, idx] = v
    return out


def cs_filter_center(x, present=None, center=(0.3, 0.7)):
    """operations.py:70-75 -- keep x where x < q_lo or x > q_hi, else 0 (NaN -> 0)."""
    qlo, qhi = nm.pandas_quantile_q(center[0]), nm.pandas_quantile_q(center[1])
    out = np.full(x.shape, np.nan)
    for d, idx in _row_iter(x, present):
        v = x[d, idx]
        clean = np.sort(v[~np.isnan(v)])
        if len(clean) == 0:
            lo = hi = np.nan
        else:
            lo = nm.percentile_linear(clean, qlo)
            hi = nm.percentile_linear(clean, qhi)
        keep = (v < lo) | (v > hi)
        out[d, idx] = np.where(keep, v, 0.0)
    return out


def _cs_reduce(x, present, fn):
    """Apply fn(v_row) -> out_row per date over present rows."""
    if present is None:
        return fn(np.asarray(x, dtype=np.float64))
    out = np.full(x.shape, np.nan)
    for d, idx in _row_iter(x, present):
        if len(idx):
            out[d, idx] = fn(x[d, idx][None, :])[0]
    return out


def cs_zscore(x, present=None):
    """operations.py:77-78 -- (x - mean) / std(ddof=0), no zero guard."""
    def f(v):
        m = nm.nanmean(v)
        s = nm.nanstd(v, 0)
        with np.errstate(all="ignore"):
            return (v - m[:, None]) / s[:, None]
    return _cs_reduce(x, present, f)


def cs_mean(x, present=None):
    """operations.py:85-86 -- skipna mean broadcast to every row of the date."""
    return _cs_reduce(x, present, lambda v: np.broadcast_to(nm.nanmean(v)[:, None], v.shape).copy())


def market_neutralize(x, present=None):
    """operations.py:171-182 -- z-score (ddof=0); sigma in {0, NaN} -> all 0."""
    def f(v):
        m = nm.nanmean(v)
        s = nm.nanstd(v, 0)
        with np.errstate(all="ignore"):
            z = (v - m[:, None]) / s[:, None]
        bad = (s == 0) | np.isnan(s)
        return np.where(bad[:, None], 0.0, z)
    return _cs_reduce(x, present, f)


def cs_bool(cond, true_value, false_value):
    """operations.py:80-84 -- np.where(condition, t, f) (elementwise)."""
    return np.where(cond, true_value, false_value).astype(np.float64)


# --------------------------------------------------------------------------- elementwise
def sign(x):
    """operations.py:88-89"""
    return np.sign(x)


def power(x, exp):
    """operations.py:91-92"""
    with np.errstate(all="ignore"):
        return np.power(x, exp)


def log(x):
    """operations.py:94-95"""
    with np.errstate(all="ignore"):
        return np.log(x)


def abs_(x):
    """operations.py:97-98"""
    return np.abs(x)


def clip(x, lower, upper):
    """operations.py:100-101 -- Series.clip (NaN preserved)."""
    return np.where(x < lower, lower, np.where(x > upper, upper, x))


# --------------------------------------------------------------------------- groups
def bucket_edges(bin_range=(0.2, 1.0, 0.2)):
    """operations.py:104-107"""
    low, up, step = bin_range
    return np.arange(low, up + 1e-8, step)


def bucket(x, bin_range=(0.2, 1.0, 0.2)):
    """operations.py:104-110 -- pd.cut(right=True, include_lowest=True) codes
    (label index, -1 for NaN/out of range)."""
    e = bucket_edges(bin_range)
    nb = len(e) - 1
    ids = np.searchsorted(e, x, side="left")
    ids = np.where(x == e[0], 1, ids)
    ok = (ids > 0) & (ids <= nb) & ~np.isnan(x)
    return np.where(ok, ids - 1, -1).astype(np.int32)


def _group_iter(x, g, present):
    for d, idx in _row_iter(x, present):
        gv = g[d, idx]
        for key in np.unique(gv[~np.isnan(gv)]):
            yield d, idx[gv == key]


def group_mean(x, g, present=None):
    """operations.py:112-122 -- per (date, group) skipna mean broadcast."""
    out = np.full(x.shape, np.nan)
    for d, idx in _group_iter(x, g, present):
        out[d, idx] = nm.nanmean(x[d, idx][None, :])[0]
    return out


def group_neutralize(x, g, present=None):
    """operations.py:124-134 -- x minus the per (date, group) skipna mean."""
    out = np.full(x.shape, np.nan)
    for d, idx in _group_iter(x, g, present):
        out[d, idx] = x[d, idx] - nm.nanmean(x[d, idx][None, :])[0]
    return out


def group_normalize(x, g, present=None):
    """operations.py:137-149 -- per (date, group) z (ddof=0); sigma in {0,NaN} -> 0."""
    out = np.full(x.shape, np.nan)
    for d, idx in _group_iter(x, g, present):
        v = x[d, idx][None, :]
        mu = nm.nanmean(v)[0]
        s = nm.nanstd(v, 0)[0]
        if s == 0 or np.isnan(s):
            out[d, idx] = 0.0
        else:
            out[d, idx] = (v[0] - mu) / s
    return out


def group_rank_normalized(x, g, present=None, method="average"):
    """operations.py:152-168 -- rank over non-NaN within (date, group), (r-1)/(n-1);
    <= 1 valid -> 0.5 for every row of the group."""
    out = np.full(x.shape, np.nan)
    for d, idx in _group_iter(x, g, present):
        v = x[d, idx]
        ok = ~np.isnan(v)
        if ok.sum() <= 1:
            out[d, idx] = 0.5
            continue
        r = nm.rank_1d(v[ok], method)
        o = np.full(len(v), np.nan)
        o[ok] = (r - 1) / (ok.sum() - 1)
        out[d, idx] = o
    return out


# --------------------------------------------------------------------------- regressions
def ts_regression_fast_long(dcode, scode, y, x, window, lag=0, rettype=2):
    """operations.py:185-246 on long arrays in input row order.

    ``x.shift(lag)`` is a global row shift (crosses symbols), rows with NaN y or x are
    dropped, rolling means run per symbol over the remaining rows, NaN results are
    dropped and the output is sorted by (date, symbol).  Returns (d, s, v).
    """
    if rettype not in (0, 1, 2, 3, 6):
        raise ValueError("rettype not implemented")
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    xs = np.full_like(x, np.nan)
    if lag > 0:
        xs[lag:] = x[:-lag]
    elif lag < 0:
        xs[:lag] = x[-lag:]
    else:
        xs[:] = x
    ok = ~np.isnan(y) & ~np.isnan(xs)
    od, os_, ov = [], [], []
    for sym in np.unique(scode[ok]):
        rows = np.nonzero(ok & (scode == sym))[0]
        gx, gy = xs[rows], y[rows]
        mx = nm.roll_mean(gx, window)
        my = nm.roll_mean(gy, window)
        ex2 = nm.roll_mean(gx ** 2, window)
        exy = nm.roll_mean(gx * gy, window)
        with np.errstate(all="ignore"):
            cov = exy - mx * my
            var_x = ex2 - mx ** 2
            beta = cov / var_x
            alpha = my - beta * mx
            fitted = alpha + beta * gx
            resid = gy - fitted
            var_y = nm.roll_mean(gy ** 2, window) - my ** 2
            r2 = cov ** 2 / (var_x * var_y)
        v = {0: resid, 1: alpha, 2: beta, 3: fitted, 6: r2}[rettype]
        keep = ~np.isnan(v)
        od.append(dcode[rows][keep]); os_.append(scode[rows][keep]); ov.append(v[keep])
    if not od:
        return np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0)
    od, os_, ov = np.concatenate(od), np.concatenate(os_), np.concatenate(ov)
    order = np.lexsort((os_, od))
    return od[order], os_[order], ov[order]


def cs_regression(y, x, present=None, rettype="resid"):
    """operations.py:248-304 -- per-date OLS on pair-valid rows (population moments)."""
    if rettype not in ("resid", "beta", "alpha", "fitted", "r2"):
        raise ValueError(f"ERROR: rettype={rettype}")
    out = np.full(x.shape, np.nan)
    for d, idx in _row_iter(x, present):
        xv, yv = x[d, idx], y[d, idx]
        ok = ~np.isnan(xv) & ~np.isnan(yv)
        if ok.sum() < 2:
            continue
        dx, dy = xv[ok], yv[ok]
        mx = nm.nanmean(dx[None, :])[0]
        my = nm.nanmean(dy[None, :])[0]
        with np.errstate(all="ignore"):
            cov = nm.nanmean(((dx - mx) * (dy - my))[None, :])[0]
            var_x = nm.nanmean(((dx - mx) ** 2)[None, :])[0]
            beta = cov / var_x
            alpha = my - beta * mx
            fitted = alpha + beta * dx
            resid = dy - fitted
            var_y = nm.nanmean(((dy - my) ** 2)[None, :])[0]
            r2 = cov ** 2 / (var_x * var_y)
        val = {"resid": resid, "fitted": fitted}.get(rettype)
        if val is None:
            val = np.full(ok.sum(), {"beta": beta, "alpha": alpha, "r2": r2}[rettype])
        o = np.full(len(idx), np.nan)
        o[ok] = val
        out[d, idx] = o
    return out
