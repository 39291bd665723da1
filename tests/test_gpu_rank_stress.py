"""GPU stress parity for the bucket-rank kernels (cs_rank, cs_winsor, cs_filter_center,
daily IC) on adversarial rows: every row length class of the launch table, heavy ties,
constant rows, sorted rows, signed zeros / infinities, NaN-only rows and a "sample trap"
row whose positional splitter samples are all equal (one bucket holds half the row, which
drives the in-bucket scans and the quantile bisection fallback).  Reference: the CPU
oracle (oracle/ops.py, oracle/metrics.py), itself pinned to the reference's golden
vectors.  Ranks and quantile outputs must be bit-exact; IC within 1e-9 relative."""
import numpy as np
import pytest

from golden_io import assert_close

pytestmark = pytest.mark.gpu

SIZES = [1, 2, 3, 7, 64, 511, 512, 513, 1500, 5000, 10000, 16384]
# rows whose ceil(A / NT) is not an instantiated EMAX (rounded up 7 -> 8, 9 -> 10, 11 -> 12,
# 13..15 -> 16 at NT = 512 / 1024): slots before the last one run past the row's end
ROUNDED = [3500, 4600, 5600, 7000, 8193, 9000, 11000, 13000]
NPAT = 12


def adversarial_rows(A, seed):
    rng = np.random.default_rng(seed)
    rows = []
    z = rng.standard_normal(A)
    rows.append(z.copy())                                            # 0 random
    rows.append(np.round(z, 0))                                      # 1 heavy ties
    rows.append(np.full(A, 0.25))                                    # 2 constant
    rows.append(np.sort(z))                                          # 3 ascending
    rows.append(np.sort(z)[::-1].copy())                             # 4 descending
    trap = rng.standard_normal(A)                                    # 5 sample trap
    pos = (np.arange(1024) * A) // 1024        # every positional sample (NT = 512 or 1024)
    trap[pos] = 0.0
    rows.append(trap)
    m = rng.standard_normal(A)                                       # 6 zeros / infs / NaN
    k = rng.random(A)
    m[k < 0.1] = 0.0
    m[(k >= 0.1) & (k < 0.2)] = -0.0
    m[(k >= 0.2) & (k < 0.25)] = np.inf
    m[(k >= 0.25) & (k < 0.3)] = -np.inf
    m[(k >= 0.3) & (k < 0.6)] = np.nan
    rows.append(m)
    rows.append(np.full(A, np.nan))                                  # 7 all NaN
    one = np.full(A, np.nan)                                         # 8 single value
    one[A // 2] = 1.5
    rows.append(one)
    ints = rng.integers(-3, 4, A).astype(float)                      # 9 int ties + NaN
    ints[rng.random(A) < 0.2] = np.nan
    rows.append(ints)
    rows.append(1.0 + np.spacing(1.0) * rng.integers(0, 50, A))      # 10 ulp spacing
    rows.append(np.exp(rng.standard_normal(A) * 50) * np.sign(z))    # 11 huge range
    return np.stack(rows)


@pytest.fixture(scope="module")
def eng():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import factormodeling_amd.engine as E
    return E, torch


@pytest.mark.parametrize("A", SIZES + ROUNDED)
def test_cs_rank_stress(eng, A):
    import oracle.ops as O
    E, torch = eng
    x = adversarial_rows(A, A)
    Xd = torch.as_tensor(x[None], device="cuda")
    for method in ("average", "min", "max"):
        got = E.cs_rank(Xd, method=method).cpu().numpy()[0]
        ref = O.cs_rank(x, method=method)
        assert_close(got.ravel(), ref.ravel(), exact=True, what=f"cs_rank[{method}] A={A}")


@pytest.mark.parametrize("A", SIZES)
def test_cs_rank_first_dense_stress(eng, A):
    """Methods 'first' / 'dense': LDS bitonic up to A = 8192, rows sorted in HBM beyond
    (fmx_cs_rank_sorted); bit-exact vs the oracle, incl. a ragged presence mask."""
    import oracle.ops as O
    E, torch = eng
    x = adversarial_rows(A, A + 3)
    Xd = torch.as_tensor(x[None], device="cuda")
    pres = (np.random.default_rng(A).random(x.shape) > 0.15).astype(np.uint8)
    pres[8] = 0
    pres[8, A // 2] = 1                                              # single-row date
    Pd = torch.as_tensor(pres, device="cuda")
    for method in ("first", "dense"):
        got = E.cs_rank(Xd, method=method).cpu().numpy()[0]
        ref = O.cs_rank(x, method=method)
        assert_close(got.ravel(), ref.ravel(), exact=True, what=f"cs_rank[{method}] A={A}")
        got = E.cs_rank(Xd, method=method, present=Pd).cpu().numpy()[0]
        ref = O.cs_rank(x, present=pres.astype(bool), method=method)
        assert_close(got.ravel(), ref.ravel(), exact=True, what=f"cs_rank[{method}] ragged A={A}")


def test_cs_rank_sorted_equals_bitonic(eng):
    """The HBM-sorted path equals the LDS bitonic path where both run (A <= 8192)."""
    import ctypes
    from factormodeling_amd import _lib
    E, torch = eng
    A = 5000
    X = torch.as_tensor(adversarial_rows(A, 9)[None].repeat(3, axis=0), device="cuda")
    F, D = X.shape[0], X.shape[1]
    for method in ("first", "dense"):
        ref = E.cs_rank(X, method=method)
        Y = torch.empty_like(X)
        nb = int(_lib.load().fmx_cs_rank_sorted_work_bytes(F, D, A))
        work = torch.empty(nb, dtype=torch.uint8, device="cuda")
        _lib.call("fmx_cs_rank_sorted", ctypes.c_void_p(X.data_ptr()), ctypes.c_void_p(Y.data_ptr()), F, D, A, A,
                  E.RANK[method], None, ctypes.c_void_p(work.data_ptr()), nb,
                  ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert np.array_equal(Y.cpu().numpy(), ref.cpu().numpy(), equal_nan=True), method


@pytest.mark.parametrize("A", SIZES + ROUNDED)
def test_cs_quantile_stress(eng, A):
    import oracle.ops as O
    E, torch = eng
    x = adversarial_rows(A, A + 1)
    Xd = torch.as_tensor(x[None], device="cuda")
    got = E.cs_quantile_op("winsor", Xd, 0.01, 0.99).cpu().numpy()[0]
    assert_close(got.ravel(), O.cs_winsor(x).ravel(), exact=True, what=f"winsor A={A}")
    got = E.cs_quantile_op("filter_center", Xd, 0.3, 0.7).cpu().numpy()[0]
    assert_close(got.ravel(), O.cs_filter_center(x).ravel(), exact=True, what=f"filter_center A={A}")


@pytest.mark.parametrize("A", [3, 7, 513, 1500, 5000, 3500, 9000])
def test_ic_daily_stress(eng, A):
    import oracle.metrics as OM
    E, torch = eng
    rows = adversarial_rows(A, A + 2)
    # IC needs finite x.  Row 10 (values within 50 ulps of 1.0) is excluded: there the
    # centred moments are dominated by the rounding of the mean itself, which scipy takes
    # from numpy's pairwise sum and the kernel from a block sum (parity not claimed for
    # such ill-conditioned rows).
    keep = np.isfinite(np.where(np.isnan(rows), 0.0, rows)).all(axis=1)
    keep[10] = False
    rows = rows[keep]
    D = rows.shape[0]
    rng = np.random.default_rng(A)
    R = 0.01 * rng.standard_normal((D, A))
    R[rng.random(R.shape) < 0.1] = np.nan
    X = rows[None]
    out = E.ic_daily(torch.as_tensor(X, device="cuda"), torch.as_tensor(R, device="cuda"), (1, 2)).cpu().numpy()
    for li, L in enumerate((1, 2)):
        for t in range(L, D):
            n, ic, ric, beta = OM.daily_stats(X[0, t - L], R[t])
            assert out[li, 0, 0, t] == n
            assert_close(out[li, 1:, 0, t], np.array([ic, ric, beta]), rtol=1e-9, atol=1e-12,
                         what=f"A={A} L={L} t={t}")


@pytest.mark.parametrize("A", [5000, 10000] + ROUNDED)
def test_cs_rank_winsor_rank2_stress(eng, A):
    """The fused rank + winsor pass (and its doubled ranks) and the ranks-only pass on the
    adversarial rows: rank / winsor bit-exact vs the oracle, doubled ranks = 2 * the
    average rank (0 for NaN) from both passes."""
    import oracle.ops as O
    E, torch = eng
    x = adversarial_rows(A, A + 5)
    keep = np.ones(len(x), bool)
    keep[6] = False                        # +-inf: fine for ranks, kept out of winsor's lerp
    x = x[keep]
    Xd = torch.as_tensor(x[None], device="cuda")
    rk = torch.empty(Xd.shape, dtype=E.RANK2_DTYPE, device="cuda")
    yr, yw = E.cs_rank_winsor(Xd, 0.01, 0.99, rank2=rk)
    assert_close(yr.cpu().numpy()[0].ravel(), O.cs_rank(x).ravel(), exact=True, what=f"rank A={A}")
    assert_close(yw.cpu().numpy()[0].ravel(), O.cs_winsor(x).ravel(), exact=True, what=f"winsor A={A}")
    from scipy.stats import rankdata
    exp = np.zeros(x.shape, np.int64)
    for d in range(len(x)):
        ok = ~np.isnan(x[d])
        if ok.any():
            exp[d, ok] = np.rint(2 * rankdata(x[d, ok], method="average")).astype(np.int64)
    got = rk.cpu().numpy()[0].astype(np.uint16).astype(np.int64)
    assert np.array_equal(got, exp), f"rank2 (fused) A={A}"
    got2 = E.cs_rank2(Xd).cpu().numpy()[0].astype(np.uint16).astype(np.int64)
    assert np.array_equal(got2, exp), f"rank2 (ranks-only) A={A}"
