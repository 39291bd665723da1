"""Exact CPU restatements of the third-party arithmetic the reference relies on.

Test infrastructure only (see oracle/__init__.py).

* ``pairwise_sum``  -- numpy's float64 ``add.reduce`` (pairwise summation with an
  8-accumulator unrolled leaf of <=128 elements; numpy 2.2.6
  ``numpy/_core/src/umath/loops_utils.h.src`` ``@TYPE@_pairwise_sum``).  Used by
  pandas ``nanops.nanmean``/``nanvar`` (``Series.mean()``/``.std()``) that the
  reference calls in cs_zscore (operations.py:77-78), cs_mean (:85-86),
  market_neutralize (:171-182), group ops (:112-168), cs_regression (:266-275).
* ``roll_sum/roll_mean/roll_var`` -- pandas 2.3.3 ``_libs/window/aggregations.pyx``
  fixed-window kernels (Kahan add/remove, Welford variance, consecutive-same-value
  guard), called by ``rolling(window).sum/mean/std`` in operations.py:6-21 and
  ts_regression_fast (:208-225).  Verified bit-exact against pandas in the
  build container (tests/test_oracle_golden.py).
* ``percentile_linear`` -- numpy ``percentile(method='linear')``
  (``_function_base_impl.py`` ``_quantile``/``_lerp``), reached from pandas
  ``Series.quantile`` (cs_winsor operations.py:64-68, cs_filter_center :70-75) and
  ``np.nanpercentile`` (composite_factor.py:171, :262).
"""
from __future__ import annotations

import numpy as np

PW_BLOCKSIZE = 128
BUFSIZE = 8192
# FAST: 1-D sums by numpy's own add.reduce -- the algorithm restated below, pinned to it
# bit-for-bit by tests/test_oracle_golden.py::test_pairwise_sum_is_numpys_sum.  Set only by
# the process pools of the full-size checks (tests/oracle_pool.py); off by default.
FAST = False


# --------------------------------------------------------------------------- pairwise sum
def pairwise_sum(a: np.ndarray) -> np.ndarray:
    """numpy float64 ``a.sum(axis=-1)`` bit-for-bit, vectorised over leading axes."""
    a = np.asarray(a, dtype=np.float64)
    if FAST and a.ndim == 1:
        return np.add.reduce(a)
    n = a.shape[-1]
    # the ufunc reduction iterates in buffer-sized chunks (8192 elements) and adds the
    # chunks' pairwise sums sequentially
    res = 0.0 + _pw(a, 0, min(n, BUFSIZE))
    for lo in range(BUFSIZE, n, BUFSIZE):
        res = res + _pw(a, lo, min(BUFSIZE, n - lo))
    return res


def _pw(a, lo, n):
    if n < 8:
        res = np.zeros(a.shape[:-1])
        for i in range(n):
            res = res + a[..., lo + i]
        return res
    if n <= PW_BLOCKSIZE:
        r = [a[..., lo + j].copy() for j in range(8)]
        i = 8
        stop = n - (n % 8)
        while i < stop:
            for j in range(8):
                r[j] = r[j] + a[..., lo + i + j]
            i += 8
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
        while i < n:
            res = res + a[..., lo + i]
            i += 1
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return _pw(a, lo, n2) + _pw(a, lo + n2, n - n2)


def nanmean(v: np.ndarray) -> np.ndarray:
    """pandas ``nanops.nanmean`` (skipna) along the last axis."""
    v = np.asarray(v, dtype=np.float64)
    mask = np.isnan(v)
    cnt = (~mask).sum(axis=-1).astype(np.float64)
    s = pairwise_sum(np.where(mask, 0.0, v))
    with np.errstate(all="ignore"):
        out = s / cnt
    return np.where(cnt == 0, np.nan, out)


def nanvar(v: np.ndarray, ddof: int) -> np.ndarray:
    """pandas ``nanops.nanvar`` two-pass variance along the last axis."""
    v = np.asarray(v, dtype=np.float64)
    mask = np.isnan(v)
    cnt = (~mask).sum(axis=-1).astype(np.float64)
    d = cnt - ddof
    bad = cnt <= ddof
    vz = np.where(mask, 0.0, v)
    with np.errstate(all="ignore"):
        avg = pairwise_sum(vz) / cnt
        sqr = (avg[..., None] - vz) ** 2
        sqr = np.where(mask, 0.0, sqr)
        res = pairwise_sum(sqr) / d
    return np.where(bad, np.nan, res)


def nanstd(v: np.ndarray, ddof: int) -> np.ndarray:
    with np.errstate(invalid="ignore"):
        return np.sqrt(nanvar(v, ddof))


def np_mean(v: np.ndarray) -> np.ndarray:
    """numpy ``ndarray.mean(axis=-1)`` (no NaN handling)."""
    v = np.asarray(v, dtype=np.float64)
    return pairwise_sum(v) / np.float64(v.shape[-1])


def np_std_ddof1(v: np.ndarray) -> np.ndarray:
    """numpy ``ndarray.std(ddof=1)`` (``_methods._var``: mean, x-mean, x*x, sum)."""
    v = np.asarray(v, dtype=np.float64)
    n = v.shape[-1]
    m = pairwise_sum(v) / np.float64(n)
    x = v - m[..., None]
    x = x * x
    with np.errstate(all="ignore"):
        return np.sqrt(pairwise_sum(x) / np.float64(max(n - 1, 0)))


# --------------------------------------------------------------------------- rolling (pandas)
def roll_sum(x: np.ndarray, w: int) -> np.ndarray:
    """pandas ``Rolling(w).sum()`` along axis 0, vectorised over trailing axes."""
    x = np.asarray(x, dtype=np.float64)
    T = x.shape[0]
    out = np.full(x.shape, np.nan)
    if T == 0:
        return out
    s = np.zeros(x.shape[1:]); ca = np.zeros_like(s); cr = np.zeros_like(s)
    n = np.zeros(x.shape[1:], dtype=np.int64); same = np.zeros_like(n); prev = x[0].copy()
    for i in range(T):
        if i >= w:
            v = x[i - w]; ok = v == v
            y = -v - cr; t = s + y
            cr = np.where(ok, t - s - y, cr); s = np.where(ok, t, s); n = n - ok
        v = x[i]; ok = v == v
        y = v - ca; t = s + y
        ca = np.where(ok, t - s - y, ca); s = np.where(ok, t, s); n = n + ok
        same = np.where(ok, np.where(v == prev, same + 1, 1), same)
        prev = np.where(ok, v, prev)
        res = np.where(same >= n, prev * n, s)
        out[i] = np.where(n >= w, res, np.nan)
    return out


def roll_mean(x: np.ndarray, w: int) -> np.ndarray:
    """pandas ``Rolling(w).mean()`` along axis 0 (Kahan add/remove, sign counts)."""
    x = np.asarray(x, dtype=np.float64)
    T = x.shape[0]
    out = np.full(x.shape, np.nan)
    if T == 0:
        return out
    s = np.zeros(x.shape[1:]); ca = np.zeros_like(s); cr = np.zeros_like(s)
    n = np.zeros(x.shape[1:], dtype=np.int64); neg = np.zeros_like(n); same = np.zeros_like(n)
    prev = x[0].copy()
    for i in range(T):
        if i >= w:
            v = x[i - w]; ok = v == v
            y = -v - cr; t = s + y
            cr = np.where(ok, t - s - y, cr); s = np.where(ok, t, s); n = n - ok
            neg = neg - (ok & np.signbit(v))
        v = x[i]; ok = v == v
        y = v - ca; t = s + y
        ca = np.where(ok, t - s - y, ca); s = np.where(ok, t, s); n = n + ok
        neg = neg + (ok & np.signbit(v))
        same = np.where(ok, np.where(v == prev, same + 1, 1), same)
        prev = np.where(ok, v, prev)
        with np.errstate(all="ignore"):
            r = s / n
        r = np.where(same >= n, prev, np.where((neg == 0) & (r < 0), 0.0,
                                               np.where((neg == n) & (r > 0), 0.0, r)))
        out[i] = np.where((n >= w) & (n > 0), r, np.nan)
    return out


def roll_var(x: np.ndarray, w: int, ddof: int = 1) -> np.ndarray:
    """pandas ``Rolling(w).var(ddof)`` along axis 0 (Welford + Kahan)."""
    x = np.asarray(x, dtype=np.float64)
    T = x.shape[0]
    out = np.full(x.shape, np.nan)
    if T == 0:
        return out
    mean = np.zeros(x.shape[1:]); ssq = np.zeros_like(mean); n = np.zeros_like(mean)
    ca = np.zeros_like(mean); cr = np.zeros_like(mean)
    same = np.zeros(x.shape[1:], dtype=np.int64); prev = x[0].copy()
    minp = max(w, 1)
    with np.errstate(all="ignore"):
        for i in range(T):
            if i >= w:
                v = x[i - w]; ok = v == v
                n1 = n - ok
                pm = mean - cr; y = v - cr; t = y - mean
                cr_new = t + mean - y
                mean_new = mean - t / n1
                ssq_new = ssq - (v - pm) * (v - mean_new)
                live = ok & (n1 != 0)
                dead = ok & (n1 == 0)
                cr = np.where(live, cr_new, cr)
                mean = np.where(live, mean_new, np.where(dead, 0.0, mean))
                ssq = np.where(live, ssq_new, np.where(dead, 0.0, ssq))
                n = n1
            v = x[i]; ok = v == v
            n1 = n + ok
            same = np.where(ok, np.where(v == prev, same + 1, 1), same)
            prev = np.where(ok, v, prev)
            pm = mean - ca; y = v - ca; t = y - mean
            ca_new = t + mean - y
            mean_new = np.where(n1 != 0, mean + t / n1, 0.0)
            ssq_new = ssq + (v - pm) * (v - mean_new)
            ca = np.where(ok, ca_new, ca)
            mean = np.where(ok, mean_new, mean)
            ssq = np.where(ok, ssq_new, ssq)
            n = n1
            res = np.where((n == 1) | (same >= n), 0.0, ssq / (n - ddof))
            out[i] = np.where((n >= minp) & (n > ddof), res, np.nan)
    return out


def zsqrt(v: np.ndarray) -> np.ndarray:
    """pandas ``zsqrt``: sqrt with negatives mapped to 0."""
    with np.errstate(invalid="ignore"):
        r = np.sqrt(v)
    return np.where(v < 0, 0.0, r)


# --------------------------------------------------------------------------- ranks / quantiles
def less_eq_counts(vals: np.ndarray):
    """For a 1-D array without NaN: (#strictly less, #equal incl. self) per element."""
    s = np.sort(vals)
    less = np.searchsorted(s, vals, side="left")
    eq = np.searchsorted(s, vals, side="right") - less
    return less, eq


def rank_1d(vals: np.ndarray, method: str = "average") -> np.ndarray:
    """pandas ``Series.rank(method)`` for NaN-free input (keep NaN semantics outside)."""
    n = len(vals)
    if n == 0:
        return np.zeros(0)
    less, eq = less_eq_counts(vals)
    if method == "average":
        return less + (eq + 1) / 2.0
    if method == "min":
        return (less + 1).astype(np.float64)
    if method == "max":
        return (less + eq).astype(np.float64)
    if method == "first":
        order = np.argsort(vals, kind="mergesort")
        r = np.empty(n)
        r[order] = np.arange(1, n + 1)
        return r
    if method == "dense":
        u = np.unique(vals)
        return (np.searchsorted(u, vals, side="left") + 1).astype(np.float64)
    raise ValueError(method)


def series_rank(x: np.ndarray, method: str = "average") -> np.ndarray:
    """pandas ``Series.rank`` (keep NaN)."""
    out = np.full(len(x), np.nan)
    m = ~np.isnan(x)
    out[m] = rank_1d(x[m], method)
    return out


def percentile_linear(clean_sorted: np.ndarray, q: float) -> float:
    """numpy ``percentile(..., method='linear')`` on a sorted NaN-free 1-D array at
    quantile fraction ``q`` (already divided by 100)."""
    n = len(clean_sorted)
    vi = (n - 1) * q
    if vi >= n - 1:                      # _get_indexes: both indexes -> -1 (last element)
        a = b = clean_sorted[-1]
        g = vi - (-1.0)
    else:
        prev = int(np.floor(vi))
        g = vi - prev
        a = clean_sorted[prev]
        b = clean_sorted[prev + 1]
    diff = b - a
    if g >= 0.5:
        return float(b - diff * (1 - g))
    return float(a + diff * g)


def pandas_quantile_q(q: float) -> float:
    """pandas ``Series.quantile(q)`` passes ``q*100`` to ``np.percentile`` which divides
    by 100 again; reproduce that rounding."""
    return float(np.true_divide(np.asarray([q]) * 100.0, 100)[0])
