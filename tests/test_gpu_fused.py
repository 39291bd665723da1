"""Fused multi-output kernels (one read of the panel, several operator outputs) are
bit-identical to the single-op kernels they replace in the benchmark step, which are
themselves pinned to the reference (tests/test_gpu_parity.py)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _panel(seed, F, D, A):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((F, D, A))
    X = np.where(rng.random(X.shape) < 0.1, np.round(X, 1), X)
    X[rng.random(X.shape) < 0.02] = np.nan
    X[0, 10:60, 3] = 0.3                       # constant run (ts_std exact 0 -> zscore NaN)
    X[1, 5:9, :] = np.nan                      # NaN block across the row
    return X


@pytest.mark.parametrize("D,A,W,WR", [(97, 700, 20, 10), (23, 129, 20, 10), (61, 300, 5, 5), (40, 65, 20, 20)])
def test_ts_set_matches_single_ops(dev, D, A, W, WR):
    import torch
    import factormodeling_amd.engine as E
    X = torch.as_tensor(_panel(D + A, 3, D, A), device=dev)
    outs = {k: torch.empty_like(X) for k in E.TS_SET}
    E.ts_set(X, outs, W, WR)
    for k in E.TS_SET:
        ref = E.ts(k, X, WR if k == "rank" else W).cpu().numpy()
        got = outs[k].cpu().numpy()
        assert np.array_equal(got, ref, equal_nan=True), k


def test_ts_set_subset_and_ragged(dev):
    import torch
    import factormodeling_amd.engine as E
    X = torch.as_tensor(_panel(5, 2, 50, 200), device=dev)
    outs = {"zscore": torch.empty_like(X), "decay": torch.empty_like(X)}
    E.ts_set(X, outs, 20, 10)
    assert np.array_equal(outs["zscore"].cpu().numpy(), E.ts("zscore", X, 20).cpu().numpy(), equal_nan=True)
    assert np.array_equal(outs["decay"].cpu().numpy(), E.ts("decay", X, 20).cpu().numpy(), equal_nan=True)
    pres = torch.as_tensor((np.random.default_rng(1).random((50, 200)) > 0.2).astype(np.uint8), device=dev)
    outs = {k: torch.empty_like(X) for k in E.TS_SET}
    E.ts_set(X, outs, 20, 10, pres)
    for k in E.TS_SET:
        ref = E.ts(k, X, 10 if k == "rank" else 20, pres).cpu().numpy()
        assert np.array_equal(outs[k].cpu().numpy(), ref, equal_nan=True), k


def _cs_panel(seed, F, D, A):
    X = _panel(seed, F, D, A)
    X[0, 2] = np.nan                           # empty row
    X[1, 3] = 0.75                             # constant row (sd 0: zscore NaN, neutralize 0)
    X[2, 4, 4:] = np.nan                       # 4 valid values (< 5: winsor identity)
    X[2, 6, 1:] = np.nan                       # a single valid value
    return X


@pytest.mark.parametrize("A", [9, 700, 5000, 10000])
def test_cs_zscore_neutralize_matches_single_ops(dev, A):
    import torch
    import factormodeling_amd.engine as E
    X = torch.as_tensor(_cs_panel(A, 3, 8, A), device=dev)
    Yz, Yn, st = E.cs_zscore_neutralize(X, with_stats=True)
    ref_z, st_ref = E.cs_moment_stats("zscore", X)
    ref_n = E.cs_moment("market_neutralize", X)
    assert np.array_equal(Yz.cpu().numpy(), ref_z.cpu().numpy(), equal_nan=True)
    assert np.array_equal(Yn.cpu().numpy(), ref_n.cpu().numpy(), equal_nan=True)
    assert np.array_equal(st.cpu().numpy(), st_ref.cpu().numpy(), equal_nan=True)


@pytest.mark.parametrize("A", [6, 700, 5000, 10000])
def test_cs_rank_winsor_matches_single_ops(dev, A):
    import torch
    import factormodeling_amd.engine as E
    X = torch.as_tensor(_cs_panel(A + 1, 3, 8, A), device=dev)
    Yr, Yw = E.cs_rank_winsor(X, 0.01, 0.99)
    assert np.array_equal(Yr.cpu().numpy(), E.cs_rank(X).cpu().numpy(), equal_nan=True)
    assert np.array_equal(Yw.cpu().numpy(), E.cs_quantile_op("winsor", X, 0.01, 0.99).cpu().numpy(), equal_nan=True)


def test_cs_fused_ragged(dev):
    import torch
    import factormodeling_amd.engine as E
    X = torch.as_tensor(_cs_panel(9, 3, 8, 400), device=dev)
    p = (np.random.default_rng(2).random((8, 400)) > 0.3).astype(np.uint8)
    p[5] = 0
    p[5, 17] = 1                               # single-row date
    pres = torch.as_tensor(p, device=dev)
    Yr, Yw = E.cs_rank_winsor(X, 0.01, 0.99, present=pres)
    assert np.array_equal(Yr.cpu().numpy(), E.cs_rank(X, present=pres).cpu().numpy(), equal_nan=True)
    assert np.array_equal(Yw.cpu().numpy(), E.cs_quantile_op("winsor", X, 0.01, 0.99, present=pres).cpu().numpy(),
                          equal_nan=True)
    Yz, Yn = E.cs_zscore_neutralize(X, present=pres)
    assert np.array_equal(Yz.cpu().numpy(), E.cs_moment("zscore", X, present=pres).cpu().numpy(), equal_nan=True)
    assert np.array_equal(Yn.cpu().numpy(), E.cs_moment("market_neutralize", X, present=pres).cpu().numpy(),
                          equal_nan=True)


def test_plan_ops_groups_the_c2_set():
    from factormodeling_amd import pipeline as PL
    stages = PL.plan_ops(PL.OPS, PL.ENGINE, True)
    assert [s for s, _ in stages] == ["ts_set:20:10", "cs_zscore_neutralize", "cs_rank_winsor"]
    assert sorted(o for _, ops in stages for o in ops) == sorted(PL.OPS)
    assert len(PL.plan_ops(PL.OPS, PL.ENGINE, False)) == len(PL.OPS)
