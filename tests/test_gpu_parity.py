"""GPU parity: the drop-in modules (HIP kernels via libfmx) against the reference's
golden vectors and against the CPU oracle.  Tolerances: bit-exact where the kernel
replicates pandas/numpy arithmetic (ranks, rolling Kahan/Welford, pairwise moments,
quantiles); otherwise |got - ref| <= 1e-9 + 1e-6 |ref| (north_star: 1e-6 relative)."""
import json
import os

import numpy as np
import pandas as pd
import pytest

from cases_ops import BUCKETS, CASES, TSREG
from golden_io import GOLDEN, assert_close, dense, dup_canon, gather, load, merge_dups, series

pytestmark = pytest.mark.gpu

RTOL, ATOL = 1e-6, 1e-9


@pytest.fixture(scope="module")
def fm():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import factormodeling_amd.composite_factor as cf
    import factormodeling_amd.factor_selector as fs
    import factormodeling_amd.operations as ops
    return ops, fs, cf


@pytest.fixture(scope="module", params=["ops_dense.npz", "ops_ragged.npz"])
def panel(request):
    st = load(request.param)
    dates = pd.to_datetime(st["dates"])
    sx = series(st, "in_x", dates, name="fx")
    sy = series(st, "in_y", dates, name="fy")
    sg = series(st, "in_g", dates, name="grp")
    return st, sx, sy, sg


def _check_series(got, st, key, exact):
    ref = st["out_" + key + "__v"]
    assert len(got) == len(ref), key
    assert np.array_equal(got.index.get_level_values(0), pd.to_datetime(st["dates"])[st["out_" + key + "__d"]]), key
    if bool(st["out_" + key + "__hasname"]):
        assert got.name == str(st["out_" + key + "__name"]), (key, got.name)
    else:
        assert got.name is None, (key, got.name)
    assert_close(got.to_numpy(dtype=np.float64), ref, rtol=RTOL, atol=ATOL, exact=exact, what=key)


@pytest.mark.parametrize("key", sorted(CASES))
def test_ops_vs_reference(fm, panel, key):
    ops = fm[0]
    st, sx, sy, sg = panel
    _, api, exact = CASES[key]
    got = api(ops, sx, sy, sg)
    _check_series(got, st, key, exact)


@pytest.mark.parametrize("lag,rt", TSREG)
def test_ts_regression_fast(fm, panel, lag, rt):
    ops = fm[0]
    st, sx, sy, sg = panel
    key = f"ts_regression_fast_5_{lag}_{rt}"
    got = ops.ts_regression_fast(sy, sx, 5, lag=lag, rettype=rt)
    _check_series(got, st, key, True)


@pytest.mark.parametrize("br", BUCKETS)
def test_bucket(fm, panel, br):
    ops = fm[0]
    st = panel[0]
    key = "bucket_%g_%g_%g" % br
    u = series(st, "in_" + key, pd.to_datetime(st["dates"]))
    b = ops.bucket(u, bin_range=br)
    assert np.array_equal(b.cat.codes.to_numpy(), st["out_" + key + "__codes"])
    assert list(b.cat.categories) == list(st["out_" + key + "__labels"])


def test_dataframe_batched(fm, panel):
    ops = fm[0]
    st, sx, sy, sg = panel
    df = pd.DataFrame({"a": sx, "b": sy, "c": -sx})
    for op, kw in (("ts_mean", {"window": 5}), ("cs_rank", {}), ("cs_zscore", {})):
        out = getattr(ops, op)(df, **kw)
        assert list(out.columns) == ["a", "b", "c"]
        for c in "abc":
            assert_close(out[c].to_numpy(), st[f"out_df_{op}_{c}__v"], exact=True, what=f"df_{op}_{c}")


def test_ts_corr_vs_pandas(fm):
    ops = fm[0]
    st = load("ts_corr_pandas.npz")
    dates = pd.to_datetime(st["dates"])
    sx, sy = series(st, "in_x", dates, name="fx"), series(st, "in_y", dates, name="fy")
    for w in (3, 5, 20):
        got = ops.ts_corr(sx, sy, w)
        assert_close(got.to_numpy(), st[f"out_ts_corr_{w}__v"], rtol=RTOL, atol=ATOL, what=f"ts_corr_{w}")


def _factor_frame(st):
    dates = pd.to_datetime(st["dates"])
    syms = list(st["syms"])
    names = list(st["names"])
    D, A, F = st["X"].shape
    idx = pd.MultiIndex.from_product([dates, syms], names=["date", "symbol"])
    df = pd.DataFrame(st["X"].reshape(D * A, F), index=idx, columns=names)
    return dates, syms, names, df, idx


def test_single_factor_metrics(fm):
    fs = fm[1]
    st = load("metrics.npz")
    dates, syms, names, df, idx = _factor_frame(st)
    ret = pd.Series(st["R"].reshape(-1), index=idx, name="log_return")
    m = fs.single_factor_metrics(df, ret)
    X = np.moveaxis(st["X"], 2, 0)
    canon = dup_canon(X, names)
    assert [canon[n] for n in m.index] == [canon[n] for n in st["out_order"]]
    assert list(m.columns) == list(st["out_cols"])
    assert_close(m.to_numpy(), st["out_vals"], rtol=RTOL, atol=ATOL, what="metrics")


def test_factor_selector(fm):
    fs = fm[1]
    man = json.load(open(os.path.join(GOLDEN, "manifest.json")))
    st = load("selector.npz")
    dates, syms, names, df, idx = _factor_frame(st)
    ret = pd.Series(st["R"].reshape(-1), index=idx, name="log_return")
    fret = pd.DataFrame(st["FR"], index=pd.DatetimeIndex(dates, name="date"), columns=names)
    X = np.moveaxis(st["X"], 2, 0)
    canon = dup_canon(X, names)
    for case in man["files"]["selector.npz"]["cases"]:
        key = case["key"]
        sel = fs.FactorSelector(df, ret, fret, window=case["window"], method=case["method"],
                                method_kwargs=case["kwargs"])
        out = sel.prepare_selection()
        assert [str(d.date()) for d in out.index] == list(st[f"out_{key}__dates"]), key
        assert out.index.name == "date" and out.columns.name == "factor"
        ref_cols = list(st[f"out_{key}__cols"])
        assert [canon[c] for c in out.columns] == [canon[c] for c in ref_cols], key
        got = merge_dups(out.to_numpy(), list(out.columns), canon)
        ref = merge_dups(st[f"out_{key}__vals"], ref_cols, canon)
        assert np.array_equal(got > 0, ref > 0), key                  # selected sets bit-exact
        assert_close(got.ravel(), ref.ravel(), rtol=1e-12, atol=0, what=key)


# ---------------------------------------------------------------------- vs the oracle
@pytest.mark.parametrize("seed", [0, 1])
def test_ops_random_vs_oracle(fm, seed):
    """Larger random panels (incl. ties, NaN runs, constant runs) vs the oracle."""
    import oracle.ops as O
    ops = fm[0]
    rng = np.random.default_rng(seed)
    D, A = 150, 700
    x = rng.standard_normal((D, A))
    x = np.where(rng.random((D, A)) < 0.3, np.round(x, 1), x)
    x[rng.random((D, A)) < 0.05] = np.nan
    x[20:60, 5] = 2.5
    dates = pd.bdate_range("2010-01-01", periods=D)
    syms = [f"Z{i:04d}" for i in range(A)]
    idx = pd.MultiIndex.from_product([dates, syms], names=["date", "symbol"])
    s = pd.Series(x.reshape(-1), index=idx, name="f")
    checks = [
        (ops.ts_mean(s, 20), O.ts_mean(x, 20), True), (ops.ts_std(s, 20), O.ts_std(x, 20), True),
        (ops.ts_zscore(s, 10), O.ts_zscore(x, 10), True), (ops.ts_rank(s, 10), O.ts_rank(x, 10), True),
        (ops.ts_sum(s, 60), O.ts_sum(x, 60), True), (ops.ts_decay(s, 20), O.ts_decay(x, 20), False),
        (ops.cs_rank(s), O.cs_rank(x), True), (ops.cs_zscore(s), O.cs_zscore(x), True),
        (ops.cs_winsor(s), O.cs_winsor(x), True), (ops.market_neutralize(s), O.market_neutralize(x), True),
        (ops.cs_filter_center(s), O.cs_filter_center(x), True),
    ]
    for k, (got, ref, exact) in enumerate(checks):
        assert_close(got.to_numpy(), ref.reshape(-1), rtol=RTOL, atol=ATOL, exact=exact, what=f"check{k}")


def test_ic_daily_vs_oracle(fm):
    """Daily IC / rank IC / beta of one factor vs the scipy-formula oracle."""
    import torch
    import factormodeling_amd.engine as E
    import oracle.metrics as OM
    rng = np.random.default_rng(7)
    F, D, A = 3, 40, 900
    X = rng.standard_normal((F, D, A))
    X[rng.random(X.shape) < 0.05] = np.nan
    X = np.where(rng.random(X.shape) < 0.1, np.round(X, 1), X)
    R = 0.01 * rng.standard_normal((D, A))
    R[rng.random(R.shape) < 0.05] = np.nan
    dev = torch.device("cuda")
    out = E.ic_daily(torch.as_tensor(X, device=dev), torch.as_tensor(R, device=dev), (1, 2)).cpu().numpy()
    for li, L in enumerate((1, 2)):
        for f in range(F):
            for t in range(L, D):
                n, ic, ric, beta = OM.daily_stats(X[f, t - L], R[t])
                assert out[li, 0, f, t] == n
                assert_close(out[li, 1:, f, t], np.array([ic, ric, beta]), rtol=1e-9, atol=1e-12, what=f"{L},{f},{t}")


def test_corr_gram_vs_oracle(fm):
    import torch
    import factormodeling_amd.engine as E
    import oracle.gram as OG
    rng = np.random.default_rng(3)
    F, D, A = 70, 12, 333
    X = rng.standard_normal((F, D, A))
    X[rng.random(X.shape) < 0.05] = np.nan
    X[5, 3] = 1.0                          # constant row -> zero
    C = E.corr_matrix(torch.as_tensor(X, device="cuda")).cpu().numpy()
    Cref = OG.corr_matrix(X)
    np.testing.assert_allclose(C, Cref, rtol=1e-10, atol=1e-12)
    order = list(rng.permutation(F))
    assert E.greedy_prune(C, order, 0.1, 10) == OG.greedy_prune(Cref, order, 0.1, 10)


def test_composite_vs_reference(fm):
    cf = fm[2]
    st = load("composite.npz")
    dates, syms, names, df, idx = _factor_frame(st)
    sels = {"all": names, "sub": [names[i] for i in (0, 1, 2, 5, 6, 7, 9, 11)]}
    for sk, sel in sels.items():
        for meth in ("zscore", "rank"):
            out = cf.composite_factor_calculation(df, sel, method=meth)
            assert out.name == "composite_factor" and out.index.equals(df.index)
            assert_close(out.to_numpy(), st[f"out_cfc_{sk}_{meth}"], rtol=RTOL, atol=ATOL, what=f"cfc_{sk}_{meth}")
    seldf = pd.DataFrame(st["sel_W"], index=pd.DatetimeIndex(pd.to_datetime(st["sel_dates"]), name="date"),
                         columns=names)
    for meth in ("zscore", "rank"):
        out = cf.weighted_composite_factor(df, seldf, method=meth)
        assert out.name == "composite_factor" and out.index.equals(df.index)
        assert_close(out.to_numpy(), st[f"out_wcf_{meth}"], rtol=RTOL, atol=ATOL, what=f"wcf_{meth}")
    with pytest.raises(ValueError):
        cf.composite_factor_calculation(df, names, method="bogus")


def test_cs_moment_stats_vs_oracle(fm):
    """Row (mean, std ddof=0) by-product of cs_zscore == numpy pairwise nanmean/nanstd."""
    import torch
    import factormodeling_amd.engine as E
    import oracle.numerics as nm
    rng = np.random.default_rng(11)
    X = rng.standard_normal((3, 17, 1000))
    X[rng.random(X.shape) < 0.05] = np.nan
    X[1, 4] = np.nan                         # empty row -> NaN stats
    X[2, 5] = 0.75                           # constant row -> sd 0
    Y, st = E.cs_moment_stats("zscore", torch.as_tensor(X, device="cuda"))
    st = st.cpu().numpy()
    with np.errstate(all="ignore"):
        mu, sd = nm.nanmean(X), nm.nanstd(X, 0)
    assert_close(st[..., 0].ravel(), mu.ravel(), exact=True, what="mean")
    assert_close(st[..., 1].ravel(), sd.ravel(), exact=True, what="sd")
    _, st2 = E.cs_moment_stats("stats", torch.as_tensor(X, device="cuda"))
    assert np.array_equal(st2.cpu().numpy(), st, equal_nan=True)


def test_corr_gram_wide_vs_oracle(fm):
    """F > 256 takes the materialised Z/M + 128x128-tile path."""
    import torch
    import factormodeling_amd.engine as E
    import oracle.gram as OG
    rng = np.random.default_rng(5)
    F, D, A = 260, 3, 150
    X = rng.standard_normal((F, D, A))
    X[rng.random(X.shape) < 0.05] = np.nan
    C = E.corr_matrix(torch.as_tensor(X, device="cuda")).cpu().numpy()
    np.testing.assert_allclose(C, OG.corr_matrix(X), rtol=1e-10, atol=1e-12)


def test_corr_gram_fused_date_range(fm):
    """Fused Gram over a date sub-range [d0, d1) equals the oracle on that slice."""
    import torch
    import factormodeling_amd.engine as E
    import oracle.gram as OG
    rng = np.random.default_rng(6)
    F, D, A = 37, 9, 401
    X = rng.standard_normal((F, D, A))
    X[rng.random(X.shape) < 0.1] = np.nan
    C = E.corr_matrix(torch.as_tensor(X, device="cuda"), 2, 7).cpu().numpy()
    np.testing.assert_allclose(C, OG.corr_matrix(X, 2, 7), rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("A", [9, 129, 2500, 4097, 5000, 8200, 10000])
def test_cs_moment_row_lengths_vs_oracle(fm, A):
    """cs_zscore / market_neutralize bit-exact at the row lengths that pick the register-
    resident kernel (numpy leaves fit 64 x 8 lanes) and the LDS kernel (longer rows)."""
    import torch
    import factormodeling_amd.engine as E
    import oracle.ops as O
    rng = np.random.default_rng(A)
    X = rng.standard_normal((2, 6, A))
    X = np.where(rng.random(X.shape) < 0.2, np.round(X, 1), X)
    X[rng.random(X.shape) < 0.02] = np.nan
    X[0, 3] = np.nan                          # empty row
    X[1, 2] = -1.25                           # constant row
    Xd = torch.as_tensor(X, device="cuda")
    for op, ref_fn in (("zscore", O.cs_zscore), ("market_neutralize", O.market_neutralize)):
        got = E.cs_moment(op, Xd).cpu().numpy()
        for f in range(2):
            with np.errstate(all="ignore"):
                ref = ref_fn(X[f])
            assert_close(got[f].ravel(), ref.ravel(), exact=True, what=f"{op} A={A}")


def test_full_sample_metrics_long_panel_vs_oracle(fm):
    """D >= 512 takes the block-per-summary window kernel: full-sample metrics vs oracle."""
    import torch
    import factormodeling_amd.engine as E
    import oracle.metrics as OM
    rng = np.random.default_rng(21)
    F, D, A = 5, 640, 120
    X = rng.standard_normal((F, D, A))
    X[rng.random(X.shape) < 0.03] = np.nan
    X[2] = X[1]                               # duplicated factor
    R = 0.01 * rng.standard_normal((D, A)) + 0.002 * X[0]
    R[rng.random(R.shape) < 0.01] = np.nan
    daily = E.ic_daily(torch.as_tensor(X, device="cuda"), torch.as_tensor(R, device="cuda"), (1,))[0]
    summ = E.ic_window(daily, [0], [D])[0].cpu().numpy()
    _, vals = OM.single_factor_metrics(X, R)
    np.testing.assert_allclose(summ[:, [0, 1, 2, 3, 6]], vals[:, [0, 1, 2, 3, 6]], rtol=1e-6, atol=1e-9)
    assert np.array_equal(summ[1], summ[2], equal_nan=True)
