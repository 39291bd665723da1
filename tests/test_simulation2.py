"""Simulation method 'linear' (portfolio_simulation.py:172-181, :250-313), the daily P&L /
turnover / cost (:748-797), the metrics' daily IC (:799-819) and linear multi-manager
books (multi_manager.py:32-81).

Golden vectors: tests/golden/sim2.npz from tests/golden/make_golden_sim2.py (the
reference run in the build container).  CPU tests pin the oracle (oracle/simulation.py);
GPU tests run the product (factormodeling_amd.portfolio_simulation / multi_manager on
libfmx) against the goldens: linear weights bit-exact (every pandas sum is a numpy
pairwise sum the kernel replicates), P&L columns within 1e-12 relative (row sums are
reduced in a different order), metrics (rounded to 0.01 by the reference) exact.
"""
import os

import numpy as np
import pandas as pd
import pytest

import oracle.simulation as OS

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "sim2.npz"))
LIN = ["lin_dense", "lin_ragged", "lin_tiny", "lin_nocap"]
PNL = LIN + ["eq_pnl"]
COLS = ["log_return", "long_return", "short_return", "long_turnover", "short_turnover", "turnover"]


def _dims(name):
    D, A, Dm, Am = (int(v) for v in GOLD[f"{name}_dims"])
    return D, A, Dm, Am


def _grid(name, key):
    D, A, Dm, Am = _dims(name)
    out = np.full((Dm, Am), np.nan)
    out[GOLD[f"{name}_{key}__d"], GOLD[f"{name}_{key}__s"]] = GOLD[f"{name}_{key}__v"]
    return out


def _present(name, key):
    D, A, Dm, Am = _dims(name)
    p = np.zeros((Dm, Am), dtype=bool)
    p[GOLD[f"{name}_{key}__d"], GOLD[f"{name}_{key}__s"]] = True
    return p


def _series(name, key):
    D, A, Dm, Am = _dims(name)
    dates = pd.bdate_range("2021-01-01", periods=Dm)
    syms = np.array([f"S{k:04d}" for k in range(A)] + [f"X{k:02d}" for k in range(Am - A)], dtype=object)
    idx = pd.MultiIndex.from_arrays([dates[GOLD[f"{name}_{key}__d"]], syms[GOLD[f"{name}_{key}__s"]]],
                                    names=["date", "symbol"])
    return pd.Series(GOLD[f"{name}_{key}__v"], index=idx)


def _same(a, b):
    return np.array_equal(a, b, equal_nan=True)


def _ref_result(key, Dm):
    d = GOLD[f"{key}_res_d"]
    v = GOLD[f"{key}_res_v"]
    return d, v


@pytest.mark.parametrize("name", LIN)
def test_oracle_linear_matches_reference(name):
    D, A, Dm, Am = _dims(name)
    X = _grid(name, "x")[:D, :A]
    pres = _present(name, "x")[:D, :A]
    W, c = OS.trade_linear(X, pres, float(GOLD[f"{name}_mw"]))
    assert _same(W, _grid(name, "w")[:D, :A])
    counts = np.zeros((D, 2))
    counts[GOLD[f"{name}_count_dates"]] = GOLD[f"{name}_counts"]
    np.testing.assert_array_equal(c, counts)


def _oracle_pnl(name, tc):
    D, A, Dm, Am = _dims(name)
    W = _grid(name, "w")
    R = _grid(name, "ret")
    CAP = _grid(name, "cap")
    wd = _present(name, "w").any(axis=1)
    rd = _present(name, "ret").any(axis=1)
    cd = _present(name, "cap").any(axis=1)
    return OS.portfolio_returns(W, wd, R, rd, CAP, cd, transaction_cost=tc)


def _check_result(keep, cols, key):
    d, v = _ref_result(key, len(keep))
    assert sorted(np.flatnonzero(keep)) == sorted(d.tolist()), key
    assert list(d) == sorted(d.tolist(), reverse=True)                # date descending
    np.testing.assert_allclose(cols[d], v, rtol=1e-12, atol=1e-15, err_msg=key)


@pytest.mark.parametrize("name", PNL)
@pytest.mark.parametrize("tc", [True, False])
def test_oracle_pnl_matches_reference(name, tc):
    keep, cols, contrib = _oracle_pnl(name, tc)
    key = f"{name}_tc{int(tc)}"
    _check_result(keep, cols, key)
    D, A, Dm, Am = _dims(name)
    syms = np.array([f"S{k:04d}" for k in range(A)] + [f"X{k:02d}" for k in range(Am - A)])
    for leg, j in (("long", 0), ("short", 1)):
        s = pd.Series(contrib[:, j], index=syms)
        top = s.nlargest(10)
        assert list(top.index) == list(GOLD[f"{key}_top_{leg}_s"]), (key, leg)
        np.testing.assert_allclose(top.to_numpy(), GOLD[f"{key}_top_{leg}_v"], rtol=1e-12, atol=1e-15)


@pytest.mark.parametrize("name", PNL)
def test_oracle_metrics_matches_reference(name):
    D, A, Dm, Am = _dims(name)
    keep, cols, _ = _oracle_pnl(name, True)
    wd = _present(name, "w").any(axis=1)
    X = _grid(name, "x")
    R = _grid(name, "ret")
    m = OS.metrics(X, R, cols[wd, 3], cols[wd, 4])
    np.testing.assert_array_equal(m, GOLD[f"{name}_metrics"])


# --------------------------------------------------------------------------------- GPU
def _settings(name, tc, contributor=True):
    from factormodeling_amd.portfolio_simulation import SimulationSettings
    ret, cap = _series(name, "ret"), _series(name, "cap")
    inv = pd.Series(1.0, index=ret.index)
    return SimulationSettings(returns=ret, cap_flag=cap, investability_flag=inv, factors_df=None,
                              method=str(GOLD[f"{name}_method"]), pct=0.15, max_weight=float(GOLD[f"{name}_mw"]),
                              plot=False, transaction_cost=tc, contributor=contributor)


@pytest.mark.gpu
@pytest.mark.parametrize("name", PNL)
def test_simulation_trade_list_on_gpu(name):
    from factormodeling_amd.portfolio_simulation import Simulation
    sim = Simulation(name="g", custom_feature=_series(name, "x"), settings=_settings(name, True))
    w, counts = sim._daily_trade_list()
    ref = _series(name, "w")
    assert w.index.equals(ref.index)
    assert _same(w.to_numpy(), ref.to_numpy())
    np.testing.assert_array_equal(counts.to_numpy(dtype=np.float64), GOLD[f"{name}_counts"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", PNL)
@pytest.mark.parametrize("tc", [True, False])
def test_simulation_portfolio_returns_on_gpu(name, tc):
    from factormodeling_amd.portfolio_simulation import Simulation
    sim = Simulation(name="g", custom_feature=_series(name, "x"), settings=_settings(name, tc))
    res, tl, ts = sim._daily_portfolio_returns(_series(name, "w"))
    key = f"{name}_tc{int(tc)}"
    D, A, Dm, Am = _dims(name)
    dates = pd.bdate_range("2021-01-01", periods=Dm)
    d, v = _ref_result(key, Dm)
    assert list(res.columns) == ["date"] + COLS
    assert list(pd.DatetimeIndex(res["date"])) == list(dates[d])
    np.testing.assert_allclose(res[COLS].to_numpy(dtype=np.float64), v, rtol=1e-12, atol=1e-15)
    assert list(tl.index) == list(GOLD[f"{key}_top_long_s"])
    np.testing.assert_allclose(tl.to_numpy(), GOLD[f"{key}_top_long_v"], rtol=1e-12, atol=1e-15)
    assert list(ts.index) == list(GOLD[f"{key}_top_short_s"])
    np.testing.assert_allclose(ts.to_numpy(), GOLD[f"{key}_top_short_v"], rtol=1e-12, atol=1e-15)


@pytest.mark.gpu
@pytest.mark.parametrize("name", PNL)
def test_simulation_metrics_on_gpu(name):
    from factormodeling_amd.portfolio_simulation import Simulation
    st = _settings(name, True)
    sim = Simulation(name="g", custom_feature=_series(name, "x"), settings=st)
    sim.custom_feature = sim.custom_feature * st.investability_flag
    w = _series(name, "w")
    counts = pd.DataFrame(GOLD[f"{name}_counts"], columns=["long_count", "short_count"])
    m = sim._calculate_metrics(w, counts)
    assert list(m.columns) == list(GOLD[f"{name}_metric_cols"])
    np.testing.assert_array_equal(m.to_numpy(dtype=np.float64).ravel(), GOLD[f"{name}_metrics"])


@pytest.mark.gpu
def test_multimanager_linear_and_late_symbol_order():
    from factormodeling_amd.multi_manager import compute_multimanager_weights
    dates = pd.to_datetime(GOLD["mm_dates"])
    idx = pd.MultiIndex.from_arrays([dates[GOLD["mm_index_date"]], GOLD["mm_index_sym"].astype(object)],
                                    names=["date", "symbol"])
    names = [f"f{k}" for k in range(GOLD["mm_X"].shape[1])]
    factors_df = pd.DataFrame(GOLD["mm_X"], index=idx, columns=names)
    fw = pd.DataFrame(GOLD["mm_fw"], index=pd.Index(dates[2:], name="date"), columns=list(GOLD["mm_fw_cols"]))
    settings = dict(method="linear", pct=0.2, max_weight=0.08)
    w, counts = compute_multimanager_weights(factors_df, fw, settings)
    assert list(w.index.get_level_values(0)) == list(dates[GOLD["mm_w_d"]])
    assert list(w.index.get_level_values(1)) == list(GOLD["mm_w_s"])            # symbol order within dates
    np.testing.assert_array_equal(w.to_numpy(), GOLD["mm_w_v"])
    np.testing.assert_array_equal(counts.to_numpy(dtype=np.float64), GOLD["mm_counts"])


@pytest.mark.gpu
@pytest.mark.parametrize("method", ["equal", "linear"])
def test_trade_list_shuffled_rows(method):
    """Row order across dates does not change the trade list (the reference groups by date
    and sorts before the per-symbol shift); a shuffled input matches the sorted one."""
    from factormodeling_amd.simulation import daily_trade_list
    s = _series("lin_ragged", "x")
    rng = np.random.default_rng(5)
    d = s.index.get_level_values(0)
    # shuffle whole dates (keeps each date's internal row order)
    udates = np.array(sorted(set(d)))
    perm = rng.permutation(len(udates))
    rank = {dt: perm[i] for i, dt in enumerate(udates)}
    order = np.argsort([rank[x] for x in d], kind="stable")
    w1, c1 = daily_trade_list(s, 0.15, method, 0.025)
    w2, c2 = daily_trade_list(s.iloc[order], 0.15, method, 0.025)
    assert w1.index.equals(w2.index)
    assert _same(w1.to_numpy(), w2.to_numpy())
    assert c1.equals(c2)
