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


@pytest.mark.parametrize("D,A,W,WR", [(97, 700, 20, 10), (23, 129, 20, 10), (61, 300, 5, 5), (40, 65, 20, 20),
                                      (200, 131, 60, 20), (400, 70, 150, 80)])
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
    for W, WR in ((20, 10), (7, 3), (45, 30)):   # ragged: the one-pass moments + rank + decay
        outs = {k: torch.empty_like(X) for k in E.TS_SET}
        E.ts_set(X, outs, W, WR, pres)
        for k in E.TS_SET:
            ref = E.ts(k, X, WR if k == "rank" else W, pres).cpu().numpy()
            assert np.array_equal(outs[k].cpu().numpy(), ref, equal_nan=True), (k, W, WR)
    outs = {"std": torch.empty_like(X)}             # a moments subset on the general path
    E.ts_set(X, outs, 33, 10)
    assert np.array_equal(outs["std"].cpu().numpy(), E.ts("std", X, 33).cpu().numpy(), equal_nan=True)


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
    assert [s for s, _ in stages] == ["ts_set:20:10", "cs_rank_winsor_zn"]
    assert sorted(o for _, ops in stages for o in ops) == sorted(PL.OPS)
    stages = PL.plan_ops(PL.OPS, PL.ENGINE, True, zn=False)
    assert [s for s, _ in stages] == ["ts_set:20:10", "cs_rank_winsor", "cs_zscore_neutralize"]
    assert sorted(o for _, ops in stages for o in ops) == sorted(PL.OPS)
    assert len(PL.plan_ops(PL.OPS, PL.ENGINE, False)) == len(PL.OPS)


@pytest.mark.parametrize("A", [9, 700, 3500, 5000, 10000, 13000])
def test_cs_rank_winsor_zn_matches_separate_passes(dev, A):
    """The four cross-sectional operators in one pass (fmx_cs_rank_winsor_zn) equal the two
    two-output passes bit for bit, the doubled ranks included: empty, constant, < 5-valid and
    single-valid rows, ties, rows whose EMAX is rounded up."""
    import torch
    import factormodeling_amd.engine as E
    X = torch.as_tensor(_cs_panel(A, 3, 9, A), device=dev)
    rk = torch.empty(X.shape, dtype=E.RANK2_DTYPE, device=dev)
    Yr, Yw, Yz, Yn = E.cs_rank_winsor_zn(X, 0.01, 0.99, rank2=rk)
    rk_ref = torch.empty_like(rk)
    Rr, Rw = E.cs_rank_winsor(X, 0.01, 0.99, rank2=rk_ref)
    Rz, Rn = E.cs_zscore_neutralize(X)
    for got, ref, what in ((Yr, Rr, "rank"), (Yw, Rw, "winsor"), (Yz, Rz, "zscore"), (Yn, Rn, "neutralize")):
        assert np.array_equal(got.cpu().numpy(), ref.cpu().numpy(), equal_nan=True), what
    assert torch.equal(rk, rk_ref)


def _ic_case(seed, F, D, A, r_nan, x_nan=0.02):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((F, D, A))
    X = np.where(rng.random(X.shape) < 0.1, np.round(X, 1), X)      # ties
    X[rng.random(X.shape) < x_nan] = np.nan
    R = 0.01 * rng.standard_normal((D, A))
    R[rng.random(R.shape) < r_nan] = np.nan
    R[-1] = np.nan                             # forward returns not yet known
    if D > 6:
        R[3, : A // 2] = np.nan                # a long E list (tile path)
        R[5, 2:] = np.nan                      # two pairs left
        X[0, 4] = 0.25                         # constant exposures
    return X, R


@pytest.mark.parametrize("A,r_nan", [(9, 0.1), (300, 0.005), (1000, 0.05), (5000, 0.005), (5000, 0.02),
                                     (5000, 0.03), (5000, 0.045), (10000, 0.005), (12000, 0.002),
                                     (12000, 0.015)])
@pytest.mark.parametrize("lags", [(1, 2), (1,), (0, 2, 5)])
def test_ic_ranked_matches_standalone_ic(dev, A, r_nan, lags):
    """Daily IC from cs_rank_winsor's doubled ranks (one wave per row, single-pass shifted
    moments; rows with long NaN-return lists through the workgroup kernel) == the
    standalone two-pass IC: pair counts exactly, statistics to 1e-12 relative."""
    import torch
    import factormodeling_amd.engine as E
    F, D = (3, 9) if A <= 5000 else (2, 8)
    X, R = _ic_case(A + len(lags), F, D, A, r_nan)
    Xt, Rt = torch.as_tensor(X, device=dev), torch.as_tensor(R, device=dev)
    rk = torch.empty(X.shape, dtype=E.RANK2_DTYPE, device=dev)
    E.cs_rank_winsor(Xt, 0.01, 0.99, rank2=rk)
    got = E.ic_daily(Xt, Rt, lags, rank2=rk).cpu().numpy()
    ref = E.ic_daily(Xt, Rt, lags).cpu().numpy()
    assert np.array_equal(got[:, 0], ref[:, 0])
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    np.testing.assert_allclose(got[:, 1:], ref[:, 1:], rtol=1e-12, atol=1e-14, equal_nan=True)


@pytest.mark.parametrize("A,r_nan", [(1, 0.0), (9, 0.1), (300, 0.005), (1000, 0.05), (5000, 0.005), (5000, 0.045),
                                     (5000, 0.07), (10000, 0.005), (12000, 0.015), (16384, 0.004)])
@pytest.mark.parametrize("lags", [(1, 2), (1,), (0, 2)])
def test_rank_winsor_ic_fused_matches_standalone(dev, A, r_nan, lags):
    """The IC fused into the rank pass (fmx_cs_rank_winsor_ic: the ranks never leave the
    workgroup; rows with > 256 NaN returns through the workgroup list kernel) == the
    standalone IC: pair counts exactly, statistics to 1e-12 relative; the rank / winsor
    outputs bit-identical to fmx_cs_rank_winsor; the ranks-only variant gives the same
    records."""
    import torch
    import factormodeling_amd.engine as E
    F, D = (3, 9) if A <= 5000 else (2, 7)
    X, R = _ic_case(A + 3 * len(lags), F, D, A, r_nan)
    if A == 1:
        X[0, 2, 0] = np.nan
    Xt, Rt = torch.as_tensor(X, device=dev), torch.as_tensor(R, device=dev)
    yr, yw, got = E.cs_rank_winsor_ic(Xt, Rt, lags)
    _, _, got2 = E.cs_rank_winsor_ic(Xt, Rt, lags, ranks_only=True)
    rr, rw = E.cs_rank_winsor(Xt, 0.01, 0.99)
    assert np.array_equal(yr.cpu().numpy(), rr.cpu().numpy(), equal_nan=True)
    assert np.array_equal(yw.cpu().numpy(), rw.cpu().numpy(), equal_nan=True)
    got, got2 = got.cpu().numpy(), got2.cpu().numpy()
    assert np.array_equal(got, got2, equal_nan=True)
    if A <= 12288:
        ref = E.ic_daily(Xt, Rt, lags).cpu().numpy()
    else:                                      # beyond the standalone kernels: the ranked IC
        rk = torch.empty(X.shape, dtype=E.RANK2_DTYPE, device=dev)
        E.cs_rank_winsor(Xt, 0.01, 0.99, rank2=rk)
        ref = E.ic_daily(Xt, Rt, lags, rank2=rk).cpu().numpy()
    assert np.array_equal(got[:, 0], ref[:, 0])
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    np.testing.assert_allclose(got[:, 1:], ref[:, 1:], rtol=1e-12, atol=1e-14, equal_nan=True)


def test_rank2_is_doubled_average_rank(dev):
    import torch
    from scipy.stats import rankdata
    import factormodeling_amd.engine as E
    X, _ = _ic_case(4, 2, 6, 777, 0.0, x_nan=0.05)
    X[1, 2] = np.nan
    X[1, 3, 1:] = np.nan                       # single valid value
    Xt = torch.as_tensor(X, device=dev)
    rk = torch.empty(X.shape, dtype=E.RANK2_DTYPE, device=dev)
    E.cs_rank_winsor(Xt, 0.01, 0.99, rank2=rk)
    got = rk.cpu().numpy().view(np.uint16)
    for f in range(2):
        for d in range(6):
            x = X[f, d]
            ok = ~np.isnan(x)
            exp = np.zeros(x.shape, dtype=np.int64)
            if ok.any():
                exp[ok] = (2 * rankdata(x[ok], method="average")).astype(np.int64)
            assert np.array_equal(got[f, d].astype(np.int64), exp), (f, d)


def test_rank2_rejects_presence_mask(dev):
    import torch
    import factormodeling_amd.engine as E
    from factormodeling_amd._lib import FmxError
    X = torch.zeros((1, 3, 10), dtype=torch.float64, device=dev)
    pres = torch.ones((3, 10), dtype=torch.uint8, device=dev)
    rk = torch.empty(X.shape, dtype=E.RANK2_DTYPE, device=dev)
    with pytest.raises(FmxError):
        E.cs_rank_winsor(X, 0.01, 0.99, present=pres, rank2=rk)


def test_step_ranked_ic_matches_unranked(dev):
    """The C2 step's IC stage through the operator set's ranks gives the same daily
    records (to 1e-12), selection and pruning as the standalone IC."""
    import torch
    from factormodeling_amd import pipeline as PL

    class Unranked(PL.EngineBackend):
        ranked_ic_max_a = 0

    class Fused(PL.EngineBackend):
        fused_ic = True

    class Unfused(PL.EngineBackend):
        fused_ic = False

    cfg = PL.StepConfig(sel_window=10)
    out = []
    for be in (Fused(), Unfused(), Unranked()):
        sp = PL.ShardedPanel(60, 400, 6, 0, 1, dev, seed=3, halo=cfg.halo)
        col = {}
        timers = []
        w, kept = PL.run_step(sp, cfg, be=be, collect=col, timers=timers)
        names = {n for n, _, _ in timers}
        out.append((col["daily"].cpu().numpy(), w.cpu().numpy(), kept, getattr(sp, "rank2", None) is not None,
                    names))
    assert out[0][3] and out[1][3] and not out[2][3]
    assert "cs_rank_winsor_ic" in out[0][4] and "ic_daily" not in out[0][4]      # fused: no IC stage
    assert "ic_daily" in out[1][4]
    for o in out[1:]:
        np.testing.assert_allclose(out[0][0], o[0], rtol=1e-12, atol=1e-14, equal_nan=True)
        assert np.array_equal(out[0][1], o[1])
        assert list(out[0][2]) == list(o[2])


def test_ic_ranked_long_rows_vs_oracle(dev):
    """A = 16384: beyond the standalone IC's LDS (it fails loudly); the ranked IC runs and
    matches the oracle's single_factor_metrics daily records."""
    import torch
    import factormodeling_amd.engine as E
    import oracle.metrics as OM
    from factormodeling_amd._lib import FmxError
    A, D = 16384, 6
    X, R = _ic_case(11, 1, D, A, 0.004)
    Xt, Rt = torch.as_tensor(X, device=dev), torch.as_tensor(R, device=dev)
    with pytest.raises(FmxError):
        E.ic_daily(Xt, Rt, (1,))
    rk = torch.empty(X.shape, dtype=E.RANK2_DTYPE, device=dev)
    E.cs_rank_winsor(Xt, 0.01, 0.99, rank2=rk)
    got = E.ic_daily(Xt, Rt, (1, 2), rank2=rk).cpu().numpy()
    for m, L in enumerate((1, 2)):
        for td in range(L, D):
            ref = OM.daily_stats(X[0, td - L], R[td])
            assert got[m, 0, 0, td] == ref[0]
            np.testing.assert_allclose(got[m, 1:, 0, td], ref[1:], rtol=1e-9, atol=1e-12, equal_nan=True)


@pytest.mark.parametrize("A", [9, 777, 5000, 10000])
def test_cs_rank2_matches_rank_winsor_ranks(dev, A):
    """The ranks-only pass (fmx_cs_rank2, the C5 IC's rank pass) writes exactly the doubled
    ranks the fused rank+winsor pass writes."""
    import torch
    import factormodeling_amd.engine as E
    X, _ = _ic_case(A + 7, 2, 6, A, 0.0, x_nan=0.05)
    X[1, 2] = np.nan                           # empty row
    X[1, 3, 1:] = np.nan                       # single valid value
    Xt = torch.as_tensor(X, device=dev)
    ref = torch.empty(X.shape, dtype=E.RANK2_DTYPE, device=dev)
    E.cs_rank_winsor(Xt, 0.01, 0.99, rank2=ref)
    got = E.cs_rank2(Xt)
    assert np.array_equal(got.cpu().numpy(), ref.cpu().numpy())


def _rank2_rows_check(A):
    """Ranks-only pass over rows of 8193..10240 assets (more rows than the grid holds), with
    heavy ties, NaN, empty and single-value rows: doubled average ranks = 2 * scipy
    rankdata(average), 0 for NaN."""
    import torch
    from scipy.stats import rankdata
    import factormodeling_amd.engine as E
    rng = np.random.default_rng(A)
    F, D = 2, 300                                # 600 rows > 256 CUs
    X = rng.standard_normal((F, D, A))
    X[:, ::3] = np.round(X[:, ::3], 1)           # tie-heavy rows
    X[:, 1::7] = np.round(X[:, 1::7] * 3)        # few distinct values
    X[rng.random(X.shape) < 0.03] = np.nan
    X[0, 5] = np.nan                             # empty row
    X[1, 9, 1:] = np.nan                         # single valid value
    X[1, 11] = 2.5                               # one value
    Xt = torch.as_tensor(X, device="cuda")
    got = E.cs_rank2(Xt).cpu().numpy().astype(np.int64)
    for f in range(F):
        for d in range(D):
            x = X[f, d]
            ok = ~np.isnan(x)
            exp = np.zeros(A, dtype=np.int64)
            if ok.any():
                exp[ok] = np.rint(2 * rankdata(x[ok], method="average")).astype(np.int64)
            assert np.array_equal(got[f, d], exp), (f, d)


@pytest.mark.parametrize("A", [8193, 10000, 10240])
def test_cs_rank2_long_rows_vs_rankdata(dev, A):
    """The default ranks-only kernel for C5-length rows (k_cs_rank_fa<1024, 10>, two rows per
    CU where the LDS allows) against scipy."""
    _rank2_rows_check(A)


def test_cs_rank2_persistent_rows_vs_rankdata(dev):
    """The persistent ranks-only kernel (k_cs_rank2_pf: one row per CU, the next row's loads
    in flight; FMX_RANK2_PF=1, read once per process: a child process) against scipy."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = ("import sys; sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + '/tests'); "
              "import test_gpu_fused as t\nfor A in (8193, 10000, 10240): t._rank2_rows_check(A)\nprint('OK')")
    env = dict(os.environ, FMX_RANK2_PF="1")
    r = subprocess.run([sys.executable, "-c", script, root], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


def test_ts_set_division_edge_values(dev):
    """The fused rolling set is bit-identical to the single-op kernels on zero / signed-zero
    / huge / subnormal-range / infinite values, exact ties and a large offset."""
    import torch
    import factormodeling_amd.engine as E
    rng = np.random.default_rng(17)
    F, D, A = 3, 120, 256
    X = rng.standard_normal((F, D, A))
    X[0, :, :64] = 0.0                                           # zero sums
    X[0, :, 64:96] = -0.0                                        # signed zeros
    X[0, :, 96:128] *= 1e300                                     # huge (sums overflow to inf)
    X[0, :, 128:160] *= 1e-308                                   # subnormal-range dividends
    X[1] = np.round(X[1] * 3) / 7.0                              # many exact ties / repeating thirds
    X[1, 30:50, :32] = np.inf
    X[1, 60:70, 32:64] = -np.inf
    X[2] = 1e8 + rng.standard_normal((D, A)) * 1e-4              # large offset, tiny spread
    X[2, rng.random((D, A)) < 0.05] = np.nan
    Xt = torch.as_tensor(X, device=dev)
    outs = {k: torch.empty_like(Xt) for k in E.TS_SET}
    E.ts_set(Xt, outs, 20, 10)
    for k in E.TS_SET:
        ref = E.ts(k, Xt, 10 if k == "rank" else 20).cpu().numpy()
        got = outs[k].cpu().numpy()
        assert np.array_equal(np.isnan(got), np.isnan(ref)), k
        assert np.array_equal(got.view(np.uint64)[~np.isnan(got)], ref.view(np.uint64)[~np.isnan(ref)]), k


def test_step_streams_match_sequential(dev):
    """The opt-in concurrent step (independent chains on their own HIP streams, separate
    output buffers per stage) gives the same operator outputs, daily records, selection
    and kept set as the sequential step."""
    from factormodeling_amd import pipeline as PL
    out = []
    for streams in (False, True):
        cfg = PL.StepConfig(sel_window=10, streams=streams)
        sp = PL.ShardedPanel(60, 400, 6, 0, 1, dev, seed=5, halo=cfg.halo)
        col = {}
        w, kept = PL.run_step(sp, cfg, collect=col)
        out.append((col, w.cpu().numpy(), list(kept)))
    a, b = out
    for k in a[0]:
        if hasattr(a[0][k], "cpu"):
            assert np.array_equal(a[0][k].cpu().numpy(), b[0][k].cpu().numpy(), equal_nan=True), k
    assert np.array_equal(a[1], b[1]) and a[2] == b[2]


@pytest.mark.parametrize("A", [700, 5000])
def test_gram_from_zscore_equals_gram_from_stats(dev, A):
    """The fused Gram from the cs_zscore output (the benchmarked step) equals the one that
    z-scores the raw panel with the row stats: same Z, same validity, same sums."""
    import factormodeling_amd.engine as E
    import torch
    X = torch.as_tensor(_cs_panel(A + 11, 5, 12, A), device=dev)
    Yz, Yn, st = E.cs_zscore_neutralize(X, with_stats=True)
    G1, N1 = E.gram_fused(X, st, 0, 12)
    G2, N2 = E.gram_fused(Yz, None, 0, 12)
    assert np.array_equal(N1.cpu().numpy(), N2.cpu().numpy())
    assert np.array_equal(G1.cpu().numpy(), G2.cpu().numpy())


@pytest.mark.parametrize("D,A,d0,d1", [(40, 700, 11, 29), (33, 5000, 21, 33), (25, 129, 0, 7), (30, 9000, 3, 30),
                                         (20, 10000, 5, 17)])
def test_date_range_entries_match_whole_panel_rows(dev, D, A, d0, d1):
    """fmx_cs_rank_winsor_zn_dates / fmx_cs_rank2_dates (the sharded step: owned dates before
    the halo lands, the halo rows' doubled ranks after): the rows of [d0, d1) bit-identical to
    the whole-panel pass, every other row untouched."""
    import torch
    import factormodeling_amd.engine as E
    X = torch.as_tensor(_panel(D * 7 + A, 3, D, A), device=dev)
    rk_full = torch.empty(X.shape, dtype=E.RANK2_DTYPE, device=dev)
    full = E.cs_rank_winsor_zn(X, rank2=rk_full)
    outs = [torch.full_like(X, 7.0) for _ in range(4)]
    rk = torch.full(X.shape, 12345, dtype=E.RANK2_DTYPE, device=dev)
    E.cs_rank_winsor_zn(X, 0.01, 0.99, *outs, rank2=rk, dates=(d0, d1))
    for got, ref in zip(outs, full):
        g, r = got.cpu().numpy(), ref.cpu().numpy()
        assert np.array_equal(g[:, d0:d1], r[:, d0:d1], equal_nan=True)
        assert (g[:, :d0] == 7.0).all() and (g[:, d1:] == 7.0).all()
    assert torch.equal(rk[:, d0:d1], rk_full[:, d0:d1])
    assert (rk[:, :d0] == 12345).all() and (rk[:, d1:] == 12345).all()
    # the halo rows' doubled ranks afterwards complete the panel
    E.cs_rank2(X, rk, dates=(0, d0))
    E.cs_rank2(X, rk, dates=(d1, D))
    assert torch.equal(rk, rk_full)


def test_overlap_step_equals_sequential_step():
    """StepConfig.overlap (the rolling set on a side stream next to the cross-sectional
    chain, every operator in its own buffer): every collected operator output, the daily IC,
    the selections, C and the kept set equal the sequential step's bit for bit."""
    import numpy as np
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from factormodeling_amd import pipeline as PL
    dev = torch.device("cuda", 0)
    D, A, F = 150, 700, 12
    res = []
    for ov in (False, True):
        cfg = PL.StepConfig(sel_window=40, overlap=ov)
        sp = PL.ShardedPanel(D, A, F, 0, 1, dev, seed=9, halo=cfg.halo)
        col = {}
        for _ in range(2):                       # the second step reuses the buffers
            col = {}
            w, kept = PL.run_step(sp, cfg, collect=col)
        torch.cuda.synchronize()
        res.append((w.cpu().numpy(), kept, {k: (v.cpu().numpy() if hasattr(v, "cpu") else v)
                                            for k, v in col.items() if v is not None}))
    (w0, k0, c0), (w1, k1, c1) = res
    assert np.array_equal(w0, w1) and k0 == k1
    assert set(c0) == set(c1)
    for k in c0:
        a, b = c0[k], c1[k]
        if isinstance(a, np.ndarray):
            assert np.array_equal(a, b, equal_nan=True), k
