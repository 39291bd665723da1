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
