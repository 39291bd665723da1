"""Helpers to read the golden fixtures (tests/golden/*.npz) into dense panels and
pandas objects.  Fixtures are plain arrays; no pickles are loaded."""
from __future__ import annotations

import os

import numpy as np
import pandas as pd

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def dense(st, key, D, A):
    """Long-format fixture series -> (x[D][A], present[D][A])."""
    d, s, v = st[key + "__d"], st[key + "__s"], st[key + "__v"]
    x = np.full((D, A), np.nan)
    p = np.zeros((D, A), dtype=bool)
    x[d, s] = v
    p[d, s] = True
    return x, p


def series(st, key, dates=None, syms=None, name=None):
    dates = pd.to_datetime(st["dates"]) if dates is None else dates
    syms = list(st["syms"]) if syms is None else syms
    d, s, v = st[key + "__d"], st[key + "__s"], st[key + "__v"]
    idx = pd.MultiIndex.from_arrays([dates[d], [syms[k] for k in s]], names=["date", "symbol"])
    return pd.Series(v, index=idx, name=name)


def gather(out, st, key):
    return out[st[key + "__d"], st[key + "__s"]]


def assert_close(got, ref, rtol=1e-6, atol=1e-9, exact=False, what=""):
    """NaN positions must match exactly; values within rtol/atol (or bit-exact)."""
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    gn, rn = np.isnan(got), np.isnan(ref)
    bad = np.nonzero(gn != rn)[0] if got.ndim == 1 else np.argwhere(gn != rn)
    assert not len(bad), f"{what}: NaN mismatch at {bad[:10]} got={got[gn != rn][:5]} ref={ref[gn != rn][:5]}"
    m = ~gn
    if exact:
        eq = (got[m] == ref[m]) | (np.isinf(ref[m]) & (got[m] == ref[m]))
        if not eq.all():
            i = np.nonzero(~eq)[0][:5]
            raise AssertionError(f"{what}: not bit-exact at {i}: got {got[m][i]!r} ref {ref[m][i]!r}")
    else:
        np.testing.assert_allclose(got[m], ref[m], rtol=rtol, atol=atol, err_msg=what)


def dup_canon(X, names):
    """Exactly duplicated factor columns have identical metrics; the reference orders
    such ties with numpy 2.x's (unstable, CPU-dependent) quicksort argsort, so parity
    is checked modulo swapping duplicates.  Returns name -> canonical name."""
    canon = {}
    F = X.shape[0]
    for i in range(F):
        canon.setdefault(names[i], names[i])
        for j in range(i + 1, F):
            if names[j] not in canon and np.array_equal(X[i], X[j], equal_nan=True):
                canon[names[j]] = names[i]
    return canon


def merge_dups(W, cols, canon):
    """Sum the weight columns of duplicated factors into their canonical column and
    return them in the canonical order of first appearance."""
    keys = []
    for c in cols:
        if canon[c] not in keys:
            keys.append(canon[c])
    out = np.zeros((W.shape[0], len(keys)))
    for j, c in enumerate(cols):
        out[:, keys.index(canon[c])] += W[:, j]
    return out
