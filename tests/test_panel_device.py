"""PanelIndex.to_device / from_device (the drop-in boundary's host <-> device conversion,
transposes and scatters done on the device since round 6) agree with the host reference
to_dense / gather bit for bit -- dense and ragged (absent rows) indexes, Series and
DataFrame inputs in both memory orders.  Runs on the CPU device (same torch code)."""
import numpy as np
import pandas as pd
import pytest
import torch

from factormodeling_amd.panel import PanelIndex


def _frame(ragged, rng):
    dates = pd.bdate_range("2020-01-01", periods=7)
    syms = [f"S{i}" for i in range(9)]
    idx = pd.MultiIndex.from_product([dates, syms], names=["date", "symbol"])
    if ragged:
        idx = idx[rng.random(len(idx)) < 0.7]
    X = rng.standard_normal((len(idx), 4))
    X[rng.random(X.shape) < 0.1] = np.nan
    return pd.DataFrame(X, index=idx, columns=list("abcd"))


@pytest.mark.parametrize("ragged", [False, True])
def test_to_device_and_back_match_host_reference(ragged):
    rng = np.random.default_rng(3 + ragged)
    df = _frame(ragged, rng)
    P = PanelIndex(df.index)
    dev = torch.device("cpu")
    for vals in (df.to_numpy(dtype=np.float64, na_value=np.nan),            # pandas' [F][n] block view
                 np.ascontiguousarray(df.to_numpy(dtype=np.float64)),       # C-contiguous [n][F]
                 df["b"].to_numpy(dtype=np.float64)):                       # a Series
        want = P.to_dense(vals)
        got = P.to_device(vals, dev).numpy()
        assert got.shape == want.shape
        assert np.array_equal(got, want, equal_nan=True)
        back = P.from_device(torch.as_tensor(want))
        assert np.array_equal(back, P.gather(want), equal_nan=True)
