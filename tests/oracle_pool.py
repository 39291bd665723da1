"""Process pool over the host's cores for the full-size checks (test infrastructure): the
oracle's per-date statistics (oracle.metrics.daily_stats) of many factor rows at once.
Workers are spawned (no GPU state crosses) and run the oracle with numerics.FAST set:
1-D pairwise sums by numpy's own add.reduce, which tests/test_oracle_golden.py pins
bit-for-bit to the restatement."""
from __future__ import annotations

import multiprocessing as mp
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_R = None


def _init(R):
    global _R
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import oracle.numerics as nm
    nm.FAST = True
    _R = R


def _daily_rows(X):
    import oracle.metrics as OM
    return np.array([OM.daily_stats(X[k], _R[k]) for k in range(X.shape[0])], dtype=np.float64)


def daily_many(X, R, workers=None):
    """X [F][T][A] exposure rows, R [T][A] the matching return rows -> [F][T][4] (n, IC,
    rank IC, beta) of oracle.metrics.daily_stats for every (factor, row)."""
    workers = workers or min(16, os.cpu_count() or 1)
    ctx = mp.get_context("spawn")
    with ctx.Pool(workers, initializer=_init, initargs=(np.ascontiguousarray(R),)) as p:
        return np.stack(p.map(_daily_rows, [np.ascontiguousarray(X[f]) for f in range(X.shape[0])]))


def window_selection(od, t_lo, i, W, thr, top_x):
    """The window metrics of day i (targets [i - W + 1, i), od's row 0 = target t_lo) for
    every factor, and the day's icir_top weights in column order (factor_selector.py:94-139,
    factor_selection_methods.py:6-26)."""
    import oracle.metrics as OM
    a, b = i - W + 1 - t_lo, i - t_lo
    F = od.shape[0]
    vals = np.empty((F, 7))
    for f in range(F):
        seg = od[f, a:b]
        ok = seg[:, 0] >= 3
        vals[f] = OM.summarize(seg[ok, 1], seg[ok, 2], seg[ok, 3])
    order = OM.nargsort_desc(vals[:, 3])
    wo = OM.icir_top(order, vals, thr, top_x)
    wf = np.zeros(F)
    wf[order] = wo
    return vals, wf
