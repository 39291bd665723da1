"""Pin the CPU oracle against golden vectors produced by the reference itself
(tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest

import oracle.composite as OC
import oracle.metrics as OM
import oracle.ops as O
from cases_ops import BUCKETS, CASES, TSREG
from golden_io import assert_close, dense, dup_canon, gather, load, merge_dups

PANELS = ["ops_dense.npz", "ops_ragged.npz"]


@pytest.fixture(scope="module", params=PANELS)
def panel(request):
    st = load(request.param)
    D, A = len(st["dates"]), len(st["syms"])
    x, p = dense(st, "in_x", D, A)
    y, _ = dense(st, "in_y", D, A)
    g, _ = dense(st, "in_g", D, A)
    return st, x, y, g, (None if p.all() else p)


@pytest.mark.parametrize("key", sorted(CASES))
def test_ops_vs_reference(panel, key):
    st, x, y, g, p = panel
    fn, _, exact = CASES[key]
    out = fn(x, y, g, p)
    ref = st["out_" + key + "__v"]
    assert np.array_equal(st["out_" + key + "__d"], st["in_x__d"])
    assert_close(gather(out, st, "out_" + key), ref, exact=exact, what=key)


@pytest.mark.parametrize("lag,rt", TSREG)
def test_ts_regression_fast_vs_reference(panel, lag, rt):
    st, x, y, g, p = panel
    key = f"out_ts_regression_fast_5_{lag}_{rt}"
    od, os_, ov = O.ts_regression_fast_long(st["in_x__d"], st["in_x__s"], st["in_y__v"], st["in_x__v"], 5, lag, rt)
    assert np.array_equal(od, st[key + "__d"]) and np.array_equal(os_, st[key + "__s"])
    assert_close(ov, st[key + "__v"], exact=True, what=key)


@pytest.mark.parametrize("br", BUCKETS)
def test_bucket_vs_reference(panel, br):
    st = panel[0]
    key = "bucket_%g_%g_%g" % br
    u = st["in_" + key + "__v"]
    codes = O.bucket(u, br)
    assert np.array_equal(codes, st["out_" + key + "__codes"])
    assert len(st["out_" + key + "__labels"]) == len(O.bucket_edges(br)) - 1


def test_dataframe_columnwise(panel):
    st, x, y, g, p = panel
    for c, arr in (("a", x), ("b", y), ("c", -x)):
        assert_close(gather(O.ts_mean(arr, 5, p), st, f"out_df_ts_mean_{c}"), st[f"out_df_ts_mean_{c}__v"], exact=True)
        assert_close(gather(O.cs_rank(arr, p), st, f"out_df_cs_rank_{c}"), st[f"out_df_cs_rank_{c}__v"], exact=True)
        assert_close(gather(O.cs_zscore(arr, p), st, f"out_df_cs_zscore_{c}"), st[f"out_df_cs_zscore_{c}__v"], exact=True)


def test_single_factor_metrics_vs_reference():
    st = load("metrics.npz")
    X = np.moveaxis(st["X"], 2, 0)                     # [F][D][A]
    order, vals = OM.single_factor_metrics(X, st["R"])
    names = list(st["names"])
    canon = dup_canon(X, names)
    assert [canon[names[k]] for k in order] == [canon[n] for n in st["out_order"]]
    assert list(st["out_cols"]) == OM.COLS
    assert_close(vals[order], st["out_vals"], rtol=1e-9, atol=1e-12, what="metrics")


def test_factor_selector_vs_reference():
    import json, os
    from golden_io import GOLDEN
    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))
    st = load("selector.npz")
    X = np.moveaxis(st["X"], 2, 0)
    names = list(st["names"])
    D = X.shape[1]
    for case in man["files"]["selector.npz"]["cases"]:
        key = case["key"]
        rows, cols, W = OM.factor_selector(X, st["R"], st["FR"], np.ones(D, bool), case["window"],
                                           case["method"], case["kwargs"])
        assert [str(st["dates"][r]) for r in rows] == list(st[f"out_{key}__dates"]), key
        canon = dup_canon(X, names)
        ref_cols = list(st[f"out_{key}__cols"])
        assert [canon[names[c]] for c in cols] == [canon[n] for n in ref_cols], key
        ref = merge_dups(st[f"out_{key}__vals"], ref_cols, canon)
        got = merge_dups(W, [names[c] for c in cols], canon)
        assert np.array_equal(got > 0, ref > 0), key               # selected sets bit-exact
        assert_close(got.ravel(), ref.ravel(), rtol=1e-12, atol=0, what=key)


def test_composite_vs_reference():
    st = load("composite.npz")
    X = np.moveaxis(st["X"], 2, 0)
    names = list(st["names"])
    sels = {"all": names, "sub": [names[i] for i in (0, 1, 2, 5, 6, 7, 9, 11)]}
    for sk, sel in sels.items():
        for meth in ("zscore", "rank"):
            out = OC.composite_factor_calculation(X, names, sel, meth)
            assert_close(out.ravel(), st[f"out_cfc_{sk}_{meth}"], rtol=1e-9, atol=1e-12, what=f"cfc_{sk}_{meth}")
    dates = list(st["dates"])
    sd = [dates.index(d) if d in dates else -1 for d in st["sel_dates"]]
    for meth in ("zscore", "rank"):
        out = OC.weighted_composite_factor(X, names, sd, st["sel_W"], meth)
        assert_close(out.ravel(), st[f"out_wcf_{meth}"], rtol=1e-9, atol=1e-12, what=f"wcf_{meth}")


def test_ts_corr_vs_pandas():
    """ts_corr has no reference counterpart; it is pinned to pandas Rolling.corr."""
    st = load("ts_corr_pandas.npz")
    D, A = len(st["dates"]), len(st["syms"])
    x, _ = dense(st, "in_x", D, A)
    y, _ = dense(st, "in_y", D, A)
    for w in (3, 5, 20):
        out = O.ts_corr(x, y, w)
        assert_close(gather(out, st, f"out_ts_corr_{w}"), st[f"out_ts_corr_{w}__v"], exact=True, what=f"ts_corr_{w}")


# ------------------------------------------------ ragged / non-contiguous (make_golden_ragged.py)
def test_single_factor_metrics_ragged_vs_reference():
    st = load("metrics_ragged.npz")
    X = np.moveaxis(st["X"], 2, 0)
    order, vals = OM.single_factor_metrics(X, st["R"], present=st["present"])
    names = list(st["names"])
    canon = dup_canon(X, names)
    assert [canon[names[k]] for k in order] == [canon[n] for n in st["out_order"]]
    assert_close(vals[order], st["out_vals"], rtol=1e-9, atol=1e-12, what="metrics_ragged")


def _selector_cases(prefix):
    import json, os
    from golden_io import GOLDEN
    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))
    return [c for c in man["files"]["selector_ragged.npz"]["cases"] if c["key"].startswith(prefix)]


@pytest.mark.parametrize("prefix", ["ragged_", "gap_"])
def test_factor_selector_ragged_vs_reference(prefix):
    st = load("selector_ragged.npz")
    names = list(st["names"])
    if prefix == "ragged_":
        X, R, pres, FR = np.moveaxis(st["X"], 2, 0), st["R"], st["present"], st["FR"]
        mask = np.ones(X.shape[1], bool)
        dates = list(st["dates"])
    else:
        X, R, pres = np.moveaxis(st["gap_X"], 2, 0), st["gap_R"], None
        mask = st["gap_fr_mask"]
        FR = np.full((X.shape[1], X.shape[0]), np.nan)
        FR[mask] = st["gap_FR"]
        dates = list(st["gap_dates"])
    canon = dup_canon(X, names)
    for case in _selector_cases(prefix):
        key = case["key"]
        rows, cols, W = OM.factor_selector(X, R, FR, mask, case["window"], case["method"], case["kwargs"],
                                           present=pres)
        assert [str(dates[r]) for r in rows] == list(st[f"out_{key}__dates"]), key
        ref_cols = list(st[f"out_{key}__cols"])
        assert [canon[names[c]] for c in cols] == [canon[n] for n in ref_cols], key
        ref = merge_dups(st[f"out_{key}__vals"], ref_cols, canon)
        got = merge_dups(W, [names[c] for c in cols], canon)
        assert np.array_equal(got > 0, ref > 0), key
        assert_close(got.ravel(), ref.ravel(), rtol=1e-12, atol=0, what=key)


def test_ts_corr_window60_vs_pandas():
    st = load("ts_corr60_pandas.npz")
    D, A = len(st["dates"]), len(st["syms"])
    x, p = dense(st, "in_x", D, A)
    y, _ = dense(st, "in_y", D, A)
    out = O.ts_corr(x, y, 60, present=p)
    assert_close(gather(out, st, "out_ts_corr_60"), st["out_ts_corr_60__v"], exact=True, what="ts_corr_60")


def test_pairwise_sum_is_numpys_sum():
    """oracle.numerics.pairwise_sum restates numpy's float64 add.reduce (128-element leaves
    with 8 accumulators, splits at multiples of 8, 8192-element buffer chunks) bit for bit:
    pinned here against numpy itself at lengths around every boundary, which is what lets
    the full-size checks' process pools (tests/oracle_pool.py) use numpy's sum directly."""
    import oracle.numerics as nm
    rng = np.random.default_rng(12)
    lens = sorted({1, 7, 8, 9, 127, 128, 129, 255, 256, 257, 1000, 4999, 5000, 8191, 8192, 8193,
                   10000, 16384, 16385, 20000} | set(rng.integers(1, 30000, 40).tolist()))
    assert not nm.FAST
    for n in lens:
        a = rng.standard_normal(n) * np.exp(rng.uniform(-30, 30, n))
        assert nm.pairwise_sum(a) == np.add.reduce(a), n
        b = a.reshape(1, -1)
        assert nm.pairwise_sum(b)[0] == np.add.reduce(a), n
