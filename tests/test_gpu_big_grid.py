"""Row kernels past the 32-bit work-item count of a 1-D grid (fmx_grid2 / fmx_blk): F * D
rows x 1024 threads above 2^32 (4.19M rows -- C4's 5.04M daily-IC rows) used to wrap and
leave every row past the wrap unwritten.  Narrow rows keep the panels small; the last rows
of the launch are checked against the oracle."""
import numpy as np
import pytest

from golden_io import assert_close

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.mark.timeout(300)
def test_ic_daily_rows_past_2_32_work_items(dev):
    import torch
    import factormodeling_amd.engine as E
    import oracle.metrics as OM
    F, D, A = 2200, 2000, 64                        # 4.4M rows (x 1024 threads > 2^32)
    g = torch.Generator(device=dev).manual_seed(3)
    X = torch.randn((F, D, A), generator=g, dtype=torch.float64, device=dev)
    R = torch.randn((D, A), generator=g, dtype=torch.float64, device=dev)
    out = E.ic_daily(X, R, (1, 2))
    torch.cuda.synchronize()
    rng = np.random.default_rng(0)
    picks = [(F - 1, D - 1), (F - 1, D - 2), (0, D - 1), (1234, 1999), (2100, 1900)]
    picks += [(int(f), int(t)) for f, t in zip(rng.integers(0, F, 6), rng.integers(1700, D, 6))]
    for f, t in picks:
        for li, L in enumerate((1, 2)):
            n, ic, ric, beta = OM.daily_stats(X[f, t - L].cpu().numpy(), R[t].cpu().numpy())
            got = out[li, :, f, t].cpu().numpy()
            assert got[0] == n, (f, t, L)
            assert_close(got[1:], np.array([ic, ric, beta]), rtol=1e-9, atol=1e-12, what=f"IC f{f} t{t} L{L}")


@pytest.mark.timeout(300)
def test_cs_rank_rows_past_2_32_work_items(dev):
    import torch
    import factormodeling_amd.engine as E
    import oracle.ops as O
    F, D, A = 4300, 2000, 64                        # 8.6M rows (x 512 threads > 2^32)
    g = torch.Generator(device=dev).manual_seed(4)
    X = torch.randn((F, D, A), generator=g, dtype=torch.float64, device=dev)
    Y = E.cs_rank(X)
    torch.cuda.synchronize()
    for f in (F - 1, F - 2, 4200, 17):
        xs = X[f, D - 40:].cpu().numpy()
        assert_close(Y[f, D - 40:].cpu().numpy().ravel(), O.cs_rank(xs).ravel(), exact=True, what=f"cs_rank f{f}")
