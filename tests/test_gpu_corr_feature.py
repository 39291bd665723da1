"""C5's fused ts_corr -> feature pass (fmx_ts_corr_feature, k_ts_corr_feat): the feature
sign(ts_corr(x, R, W)) * x / ts_std(x, W) bit-identical to the two-pass path (fmx_ts_corr +
fmx_ts_corr_vol_feature) and to the oracle (oracle/ops.py corr_vol_feature), the optional
corr output bit-identical to fmx_ts_corr, on panels with NaN in x and in the returns,
infinities, constant windows and exact zeros."""
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


def _panel(F, D, A, seed):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((F, D, A))
    X[rng.random(X.shape) < 0.03] = np.nan
    X[0, 10:40, :5] = 1.25                        # constant windows: std 0 -> NaN feature
    X[0, :, 5] = 0.0                              # exact zeros
    X[1 % F, 50, 6:9] = np.inf
    if F >= 5:                                    # extreme exponents: the sign-only fast path's
        X[2] *= 1e-200                            # guards (|num| < 2^-500, vx vy > 2^501) send
        X[3] *= 1e150                             # these to the full num / sqrt(vx vy)
    R = 0.01 * rng.standard_normal((D, A))
    R[rng.random(R.shape) < 0.05] = np.nan
    R[30:33, 10:14] = np.nan                      # return gaps inside the window
    R[70, 15] = -np.inf
    return X, R


@pytest.mark.parametrize("W", [3, 15, 60])
def test_corr_feature_equals_two_pass(dev, W):
    import torch
    import factormodeling_amd.engine as E
    F, D, A = 5, 150, 131                         # A not a multiple of 64, F not of 4
    X, R = _panel(F, D, A, W)
    Xt, Rt = torch.as_tensor(X, device=dev), torch.as_tensor(R, device=dev)
    C = E.ts_corr(Xt, Rt, W)
    ref = E.corr_vol_feature(Xt, C, W)
    corr = torch.empty_like(Xt)
    got = E.corr_feature(Xt, Rt, W, corr_out=corr)
    assert np.array_equal(got.cpu().numpy(), ref.cpu().numpy(), equal_nan=True)
    assert np.array_equal(corr.cpu().numpy(), C.cpu().numpy(), equal_nan=True)
    got2 = E.corr_feature(Xt, Rt, W)             # no corr output
    assert np.array_equal(got2.cpu().numpy(), ref.cpu().numpy(), equal_nan=True)


def test_corr_feature_vs_oracle(dev):
    import torch
    import oracle.ops as O
    import factormodeling_amd.engine as E
    F, D, A = 3, 120, 70
    X, R = _panel(F, D, A, 7)
    X[np.isinf(X)] = 2.0                          # the oracle's restatement is for finite x
    R[np.isinf(R)] = 0.01
    got = E.corr_feature(torch.as_tensor(X, device=dev), torch.as_tensor(R, device=dev), 20).cpu().numpy()
    for f in range(F):
        assert_close(got[f].ravel(), O.corr_vol_feature(X[f], R, 20).ravel(), exact=True, what=f"feature f{f}")


def test_long_window_takes_two_pass_path(dev):
    """windows past the fused pass's table (engine.CORR_FEATURE_MAX_W) run
    ts_corr + corr_vol_feature in the pipeline instead of raising.  The limit is lowered
    on a backend instance so a small panel crosses it; both paths give the same bits."""
    import torch
    from factormodeling_amd import pipeline as PL
    import factormodeling_amd.engine as E
    D, A, F = 80, 130, 6
    cfg = PL.workload_config("c5")
    cfg.sel_window, cfg.factor_chunk, cfg.ret_ops = 20, 4, [("corr_vol", 15)]
    cfg.select = cfg.composite = False
    sp = PL.ShardedPanel(D, A, F, 0, 1, dev, seed=4, halo=cfg.halo)

    class TwoPass(PL.EngineBackend):
        corr_feature_max_w = 10

    PL.run_ret_ops(sp, cfg, be=TwoPass())
    two = sp.feature.clone()
    sp.feature = None
    PL.run_ret_ops(sp, cfg)
    torch.cuda.synchronize()
    assert np.array_equal(two.cpu().numpy(), sp.feature.cpu().numpy(), equal_nan=True)
    assert 15 <= E.CORR_FEATURE_MAX_W
