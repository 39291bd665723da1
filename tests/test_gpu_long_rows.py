"""Rows past the fine-bucket kernels' 16,384 assets and groups past the per-group LDS
sort's 8192 members (operations.py:54-68, :70-75, :152-168): the rows
are sorted in HBM (csrc/rank_sort.hip) and walked one wave per row.

* cs_rank, every method, at A = 20,000 (dense and with absent cells) vs the oracle;
* cs_winsor / cs_filter_center / the fused cs_rank + cs_winsor call at A = 20,000;
* group_rank_normalized with one group of 9,000 members (A = 10,000) and at A = 20,000;
* the sorted kernels on short rows agree bit-for-bit with the fine-bucket kernels, which
  the golden tests pin to the reference.
Bit-exact: ranks and order statistics are exact integer / selection arithmetic."""
import numpy as np
import pytest

from golden_io import assert_close

pytestmark = pytest.mark.gpu

METHODS = ["average", "min", "max", "first", "dense"]


@pytest.fixture(scope="module")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _rows(seed, D, A, nan=0.02):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((D, A))
    x = np.where(rng.random(x.shape) < 0.3, np.round(x, 1), x)      # heavy ties
    x[rng.random(x.shape) < nan] = np.nan
    x[1] = np.nan                                                     # all-NaN date
    x[2, 1:] = np.nan                                                 # one valid value
    x[3, : A // 3] = 0.5                                              # a long tie run
    return x


@pytest.mark.parametrize("method", METHODS)
def test_cs_rank_20000_assets(dev, method):
    import torch
    import factormodeling_amd.engine as E
    import oracle.ops as O
    A = 20000
    x = _rows(7, 5, A)
    got = E.cs_rank(torch.as_tensor(x[None], device=dev), method).cpu().numpy()[0]
    assert_close(got.ravel(), O.cs_rank(x, method=method).ravel(), exact=True, what=f"cs_rank {method} A={A}")


def test_cs_rank_20000_assets_with_absent_cells(dev):
    import torch
    import factormodeling_amd.engine as E
    import oracle.ops as O
    A = 20000
    x = _rows(8, 4, A)
    p = (np.random.default_rng(3).random((4, A)) > 0.25).astype(np.uint8)
    p[0] = 0
    p[0, 5] = 1                                                       # one-row date -> 0.5
    xt, pt = torch.as_tensor(x[None], device=dev), torch.as_tensor(p, device=dev)
    for method in ("average", "first"):
        got = E.cs_rank(xt, method, present=pt).cpu().numpy()[0]
        assert_close(got.ravel(), O.cs_rank(x, present=p.astype(bool), method=method).ravel(), exact=True,
                     what=f"cs_rank {method} absent")


def test_sorted_rank_matches_fine_kernels_on_short_rows(dev):
    """fmx_cs_rank_sorted == the fine-bucket / bitonic kernels at A = 3000, every method
    including scipy 'average' with NaN propagation (composites)."""
    import torch
    import factormodeling_amd.engine as E
    from factormodeling_amd import _lib
    from factormodeling_amd._lib import RANK, call, ptr, stream_ptr
    x = _rows(9, 6, 3000)
    x[4] = np.round(np.random.default_rng(1).standard_normal(3000), 1)    # no NaN: propagate ranks it
    xt = torch.as_tensor(x[None], device=dev)
    F, D, A = xt.shape
    for method in METHODS + ["scipy_average"]:
        ref = E.cs_rank(xt, method).cpu().numpy()
        y = torch.empty_like(xt)
        nb = int(_lib.load().fmx_cs_rank_sorted_work_bytes(F, D, A))
        work, wb = E._workspace_bytes(xt.device, nb)
        call("fmx_cs_rank_sorted", ptr(xt), ptr(y), F, D, A, A, RANK[method], None, ptr(work), wb, stream_ptr())
        assert np.array_equal(y.cpu().numpy(), ref, equal_nan=True), method


@pytest.mark.parametrize("A", [3000, 20000])
def test_winsor_filter_center_long_rows(dev, A):
    import torch
    import factormodeling_amd.engine as E
    import oracle.ops as O
    x = _rows(11, 5, A)
    x[4, 4:] = np.nan                                                 # 4 valid: winsor identity
    xt = torch.as_tensor(x[None], device=dev)
    got = E.cs_quantile_op("winsor", xt, 0.01, 0.99).cpu().numpy()[0]
    assert_close(got.ravel(), O.cs_winsor(x).ravel(), exact=True, what=f"winsor A={A}")
    got = E.cs_quantile_op("filter_center", xt, 0.3, 0.7).cpu().numpy()[0]
    assert_close(got.ravel(), O.cs_filter_center(x).ravel(), exact=True, what=f"filter_center A={A}")
    if A > E.FINE_RANK_MAX_A:
        yr, yw = E.cs_rank_winsor(xt, 0.01, 0.99)
        assert_close(yr.cpu().numpy()[0].ravel(), O.cs_rank(x).ravel(), exact=True, what="rank_winsor rank")
        assert_close(yw.cpu().numpy()[0].ravel(), O.cs_winsor(x).ravel(), exact=True, what="rank_winsor winsor")


@pytest.mark.parametrize("A,big", [(10000, 9000), (20000, 15000)])
@pytest.mark.parametrize("method", METHODS)
def test_group_rank_big_groups(dev, A, big, method):
    """group_rank_normalized with a (date, group) of more than 8192 members and on rows
    past 16,384 assets: rows sorted by (group, value) in HBM, vs the oracle."""
    import torch
    import factormodeling_amd.engine as E
    import oracle.ops as O
    rng = np.random.default_rng(A + len(method))
    D = 4
    x = _rows(A, D, A, nan=0.03)
    g = rng.integers(0, 7, size=(D, A)).astype(np.float64)
    g[rng.random(g.shape) < 0.01] = np.nan                            # no group -> NaN
    g[0, :big] = np.where(np.isnan(g[0, :big]), np.nan, 2.0)         # one big group on date 0
    g[3, 100:140] = 5.0
    g[3, 140:] = np.where(g[3, 140:] == 5.0, 4.0, g[3, 140:])
    x[3, 100:139] = np.nan                                            # a group with one valid member
    codes = np.where(np.isnan(g), -1, g).astype(np.int32)
    got = E.group_op("rank", torch.as_tensor(x[None], device=dev), torch.as_tensor(codes, device=dev), 7,
                     method).cpu().numpy()[0]
    ref = O.group_rank_normalized(x, g, method=method)
    assert_close(got.ravel(), ref.ravel(), exact=True, what=f"group rank {method} A={A}")


def _ic_case(seed, F, D, A):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((F, D, A))
    X[rng.random(X.shape) < 0.02] = np.nan
    X = np.where(rng.random(X.shape) < 0.3, np.round(X, 1), X)        # heavy ties
    X[1, 2] = 0.75                                                   # a constant row: IC NaN
    X[0, 3, 3:] = np.nan                                             # < 3 pairs
    R = 0.01 * rng.standard_normal((D, A)) + 0.002 * np.nan_to_num(X[0])
    R[rng.random(R.shape) < 0.03] = np.nan
    R[4] = np.nan                                                    # a date with no returns
    return X, R


def test_ic_daily_20000_assets(dev):
    """the daily IC (factor_selector.py:36-48) past 16,384 assets, from
    rows sorted in HBM (fmx_ic_daily_sorted) vs the oracle's scipy restatement."""
    import torch
    import factormodeling_amd.engine as E
    import oracle.metrics as OM
    F, D, A = 3, 7, 20000
    X, R = _ic_case(29, F, D, A)
    out = E.ic_daily(torch.as_tensor(X, device=dev), torch.as_tensor(R, device=dev), (1, 2)).cpu().numpy()
    for li, L in enumerate((1, 2)):
        for f in range(F):
            for t in range(D):
                if t < L:
                    assert out[li, 0, f, t] == 0 and np.isnan(out[li, 1:, f, t]).all()
                    continue
                n, ic, ric, beta = OM.daily_stats(X[f, t - L], R[t])
                assert out[li, 0, f, t] == n
                assert_close(out[li, 1:, f, t], np.array([ic, ric, beta]), rtol=1e-9, atol=1e-12,
                             what=f"{L},{f},{t}")


def test_ic_sorted_rows_match_wave_kernels_on_short_rows(dev):
    """The sorted-row IC and the fine / wave kernels (pinned to the reference's goldens)
    give the same records on short rows: counts exact, statistics to 1e-12."""
    import torch
    import factormodeling_amd.engine as E
    X, R = _ic_case(31, 4, 9, 700)
    Xd, Rd = torch.as_tensor(X, device=dev), torch.as_tensor(R, device=dev)
    a = E.ic_daily(Xd, Rd, (1, 2), sorted_rows=True).cpu().numpy()
    b = E.ic_daily(Xd, Rd, (1, 2), sorted_rows=False).cpu().numpy()
    assert np.array_equal(a[:, 0], b[:, 0])
    assert_close(a[:, 1:].ravel(), b[:, 1:].ravel(), rtol=1e-12, atol=1e-14, what="sorted vs wave IC")


@pytest.mark.parametrize("op", ["mean", "neutralize", "normalize"])
@pytest.mark.parametrize("A,ragged", [(20000, False), (20000, True), (700, False)])
def test_group_moments_long_rows(dev, op, A, ragged):
    """group_mean / group_neutralize / group_normalize past 16,384
    assets (fmx_group_op_long: members compacted in HBM scratch, numpy pairwise sums), bit-
    exact vs the oracle; on a short row the long-row kernel equals fmx_group_op bit for bit."""
    import torch
    import factormodeling_amd.engine as E
    import oracle.ops as O
    rng = np.random.default_rng(A + len(op) + ragged)
    D = 4
    x = _rows(A + 1, D, A, nan=0.03)
    g = rng.integers(0, 11, size=(D, A)).astype(np.float64)
    g[rng.random(g.shape) < 0.01] = np.nan
    g[1, :] = np.where(np.isnan(g[1]), np.nan, 3.0)                  # one group holds the whole row
    x[2, g[2] == 6.0] = 0.25                                          # a constant group: sigma 0 -> 0
    codes = np.where(np.isnan(g), -1, g).astype(np.int32)
    p = None
    if ragged:
        p = np.random.default_rng(5).random((D, A)) > 0.2
    pt = None if p is None else torch.as_tensor(p.astype(np.uint8), device=dev)
    xt, gt = torch.as_tensor(x[None], device=dev), torch.as_tensor(codes, device=dev)
    got = E.group_op(op, xt, gt, 11, present=pt, long_rows=True).cpu().numpy()[0]
    ref = getattr(O, "group_" + op)(x, g, p)
    assert_close(got.ravel(), ref.ravel(), exact=True, what=f"group_{op} A={A}")
    if A <= 16384:
        short = E.group_op(op, xt, gt, 11, present=pt, long_rows=False).cpu().numpy()[0]
        assert np.array_equal(got, short, equal_nan=True)


@pytest.mark.parametrize("A,ragged", [(20000, False), (20000, True), (26000, False)])
def test_trade_equal_long_rows(dev, A, ragged):
    """Trade list 'equal' past 16,384 assets (LDS-staged row up to ~19,400, re-read from
    HBM beyond) vs the oracle, bit-exact."""
    import torch
    import factormodeling_amd.engine as E
    import oracle.simulation as OS
    rng = np.random.default_rng(A)
    D = 5
    X = rng.standard_normal((D, A))
    X[rng.random(X.shape) < 0.02] = np.nan
    X[2] = np.abs(X[2])                                               # flat day
    X[3] = rng.integers(-2, 3, A).astype(np.float64)                  # tie blocks at the k-th value
    present = rng.random((D, A)) >= 0.1 if ragged else np.ones((D, A), dtype=bool)
    pres = torch.as_tensor(present.astype(np.uint8), device=dev) if ragged else None
    got, c = E.trade_equal(torch.as_tensor(X, device=dev), 0.1, present=pres)
    want, wc = OS.trade_equal(X, present, 0.1)
    assert np.array_equal(got.cpu().numpy(), want, equal_nan=True)
    np.testing.assert_array_equal(c.cpu().numpy(), wc)


@pytest.mark.parametrize("A,ragged", [(20000, False), (20000, True)])
def test_trade_linear_long_rows(dev, A, ragged):
    """Trade list 'linear' (normalised legs + cap-and-redistribute) past 16,384 assets
    (k_trade_linear_xl: the row in HBM) vs the oracle's numpy-pairwise restatement, bit-exact."""
    import torch
    import factormodeling_amd.engine as E
    import oracle.simulation as OS
    rng = np.random.default_rng(A + 1)
    D = 4
    X = rng.standard_normal((D, A))
    X[rng.random(X.shape) < 0.02] = np.nan
    X[1] = np.abs(X[1])                                               # flat day
    X[2, :40] = 50.0                                                  # a few huge signals: capped
    present = rng.random((D, A)) >= 0.1 if ragged else np.ones((D, A), dtype=bool)
    pres = torch.as_tensor(present.astype(np.uint8), device=dev) if ragged else None
    mw = 0.0005
    got, c = E.trade_linear(torch.as_tensor(X, device=dev), mw, present=pres)
    want, wc = OS.trade_linear(X, present, mw)
    assert np.array_equal(got.cpu().numpy(), want, equal_nan=True)
    np.testing.assert_array_equal(c.cpu().numpy(), wc)
