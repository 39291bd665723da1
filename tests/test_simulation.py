"""Simulation._daily_trade_list, method 'equal' (portfolio_simulation.py:96-170).

Golden vectors: tests/golden/sim.npz, made by tests/golden/make_golden_sim.py running the
reference.  CPU tests pin the oracle (oracle/simulation.py) to them; GPU tests check the
k_trade_equal + ts-delay path against both, bit-exact (continuous values: no exact ties at
the k-th value, where the reference's quicksort order is implementation-defined).
"""
import os

import numpy as np
import pandas as pd
import pytest

import oracle.simulation as OS

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "sim.npz"))
CASES = ["dense", "ragged", "small"]


def _case(name):
    D, A = (int(v) for v in GOLD[f"{name}_dims"])
    def dense(key):
        out = np.full((D, A), np.nan)
        out[GOLD[key + "__d"], GOLD[key + "__s"]] = GOLD[key + "__v"]
        return out
    present = np.zeros((D, A), dtype=bool)
    present[GOLD[f"{name}_x__d"], GOLD[f"{name}_x__s"]] = True
    counts = np.zeros((D, 2))
    counts[GOLD[f"{name}_count_dates"]] = GOLD[f"{name}_counts"]
    return dense(f"{name}_x"), present, dense(f"{name}_w"), counts, float(GOLD[f"{name}_pct"])


def _series(name):
    D, A = (int(v) for v in GOLD[f"{name}_dims"])
    dates = pd.bdate_range("2021-01-01", periods=D)
    syms = np.array([f"S{k:04d}" for k in range(A)], dtype=object)
    idx = pd.MultiIndex.from_arrays([dates[GOLD[f"{name}_x__d"]], syms[GOLD[f"{name}_x__s"]]],
                                    names=["date", "symbol"])
    return pd.Series(GOLD[f"{name}_x__v"], index=idx)


def _same(a, b):
    return np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference_golden(name):
    X, present, W, counts, pct = _case(name)
    got, c = OS.trade_equal(X, present, pct)
    assert _same(got, W)
    np.testing.assert_array_equal(c, counts)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_trade_equal_kernel_matches_golden(name):
    import torch

    import factormodeling_amd.engine as E
    X, present, W, counts, pct = _case(name)
    dev = torch.device("cuda", 0)
    pres = None if present.all() else torch.as_tensor(present.astype(np.uint8), device=dev)
    got, c = E.trade_equal(torch.as_tensor(X, device=dev), pct, present=pres)
    assert _same(got.cpu().numpy(), W)
    np.testing.assert_array_equal(c.cpu().numpy(), counts)


@pytest.mark.gpu
@pytest.mark.parametrize("D,A,pct,ragged", [(40, 5000, 0.1, False), (30, 10000, 0.05, True),
                                            (12, 3, 0.5, False), (8, 16384, 0.1, False),
                                            (10, 50, 1.5, False)])
def test_trade_equal_kernel_matches_oracle(D, A, pct, ragged):
    import torch

    import factormodeling_amd.engine as E
    rng = np.random.default_rng(D * A)
    X = rng.standard_normal((D, A))
    X[rng.random(X.shape) < 0.02] = np.nan
    X[rng.random(X.shape) < 0.02] = 0.0
    X[2] = np.abs(X[2])  # flat day
    X[3, : A // 2] = np.round(X[3, : A // 2], 1)  # many exact ties, some at the k-th value
    X[4] = rng.integers(-2, 3, A).astype(np.float64)  # discrete signal: a tie block of ~A/5 at the k-th
    present = rng.random((D, A)) >= 0.1 if ragged else np.ones((D, A), dtype=bool)
    dev = torch.device("cuda", 0)
    pres = torch.as_tensor(present.astype(np.uint8), device=dev) if ragged else None
    got, c = E.trade_equal(torch.as_tensor(X, device=dev), pct, present=pres)
    want, wc = OS.trade_equal(X, present, pct)
    assert _same(got.cpu().numpy(), want)
    np.testing.assert_array_equal(c.cpu().numpy(), wc)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_daily_trade_list_series_matches_reference(name):
    from factormodeling_amd.simulation import daily_trade_list
    s = _series(name)
    D, A = (int(v) for v in GOLD[f"{name}_dims"])
    shifted, counts = daily_trade_list(s, pct=float(GOLD[f"{name}_pct"]))
    assert shifted.index.is_monotonic_increasing and len(shifted) == len(s)
    dates = pd.bdate_range("2021-01-01", periods=D)
    syms = np.array([f"S{k:04d}" for k in range(A)], dtype=object)
    ref_idx = pd.MultiIndex.from_arrays([dates[GOLD[f"{name}_w__d"]], syms[GOLD[f"{name}_w__s"]]],
                                        names=["date", "symbol"])
    ref = pd.Series(GOLD[f"{name}_w__v"], index=ref_idx)
    pd.testing.assert_series_equal(shifted, ref, check_exact=True)
    np.testing.assert_array_equal(counts.to_numpy(), GOLD[f"{name}_counts"])
    assert list(counts.columns) == ["long_count", "short_count"]
