"""multi_manager.compute_multimanager_weights with equal-weight managers (multi_manager.py:
32-81).  Golden: tests/golden/mm.npz from tests/golden/make_golden_mm.py (runs the
reference).  CPU: the numpy fold (oracle/simulation.py) reproduces it; GPU: k_trade_equal
per manager + k_mm_combine reproduce it bit-exactly."""
import os

import numpy as np
import pandas as pd
import pytest

import oracle.simulation as OS

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "mm.npz"))
D, A = int(G["D"]), int(G["A"])
DATES = pd.bdate_range("2022-03-01", periods=D)
SYMS = np.array([f"S{k:03d}" for k in range(A)], dtype=object)
NAMES = [f"f{k}" for k in range(G["X"].shape[1])]
FW_COLS = [str(c) for c in G["fw_cols"]]


def _frames():
    idx = pd.MultiIndex.from_product([DATES, SYMS], names=["date", "symbol"])
    factors_df = pd.DataFrame(G["X"], index=idx, columns=NAMES)
    fw = pd.DataFrame(G["fw"], index=pd.Index(DATES[G["fw_dates"]], name="date"), columns=FW_COLS)
    return factors_df, fw


def _ref_weights():
    w = np.zeros((len(G["fw_dates"]), A))
    row = pd.Index(G["fw_dates"]).get_indexer(G["w_d"])
    w[row, G["w_s"]] = G["w_v"]
    return w


def test_oracle_fold_matches_reference_golden():
    factors_df, fw = _frames()
    X = G["X"].T.reshape(len(NAMES), D, A)
    colmap = [NAMES.index(c) if c in NAMES else -1 for c in FW_COLS]
    out, cnt = OS.mm_weights(X, np.ones((D, A), dtype=bool), G["fw"], colmap, G["fw_dates"], float(G["pct"]))
    np.testing.assert_array_equal(out, _ref_weights())
    np.testing.assert_array_equal(cnt, G["counts"])


@pytest.mark.gpu
def test_compute_multimanager_weights_matches_reference():
    from factormodeling_amd.multi_manager import compute_multimanager_weights
    factors_df, fw = _frames()
    w, counts = compute_multimanager_weights(factors_df, fw, {"method": "equal", "pct": float(G["pct"])})
    ref_idx = pd.MultiIndex.from_arrays([DATES[G["w_d"]], SYMS[G["w_s"]]], names=["date", "symbol"])
    pd.testing.assert_series_equal(w, pd.Series(G["w_v"], index=ref_idx), check_exact=True)
    np.testing.assert_array_equal(counts.to_numpy(), G["counts"])
    assert list(counts.columns) == ["long_count", "short_count"] and counts.index.name == "date"


# ----------------------------------------------------------------------------- MVO managers
# tests/golden/mm_mvo.npz (make_golden_mm_mvo.py): the reference's compute_multimanager_weights
# with 'mvo' managers (scipy SLSQP path, cvxpy stubbed), each manager's book, and the inputs.
GM = np.load(os.path.join(os.path.dirname(__file__), "golden", "mm_mvo.npz"))
DM, AM = int(GM["D"]), int(GM["A"])
DATES_M = pd.bdate_range("2022-06-01", periods=DM)
SYMS_M = np.array([f"M{k:02d}" for k in range(AM)], dtype=object)
NAMES_M = [f"f{k}" for k in range(GM["X"].shape[1])]


def _mvo_frames(settings_cls):
    idx = pd.MultiIndex.from_product([DATES_M, SYMS_M], names=["date", "symbol"])
    factors_df = pd.DataFrame(GM["X"], index=idx, columns=NAMES_M)
    fw = pd.DataFrame(GM["fw"], index=pd.Index(DATES_M[GM["fw_dates"]], name="date"),
                      columns=[str(c) for c in GM["fw_cols"]])
    settings = settings_cls(returns=pd.Series(GM["R"], index=idx, name="ret"), cap_flag=pd.Series(GM["CAP"], index=idx),
                            investability_flag=pd.Series(1.0, index=idx), factors_df=factors_df, method="mvo",
                            use_cvxpy=False, lookback_period=5, plot=False)
    return factors_df, fw, settings


def _golden_book(fac):
    idx = pd.MultiIndex.from_arrays([DATES_M[GM[f"book_{fac}__d"]], SYMS_M[GM[f"book_{fac}__s"]]],
                                    names=["date", "symbol"])
    w = pd.Series(GM[f"book_{fac}__v"], index=idx)
    c = pd.DataFrame(GM[f"book_{fac}__c"], columns=["long_count", "short_count"],
                     index=pd.Index(DATES_M[GM[f"book_{fac}__cd"]], name="date"))
    return w, c


@pytest.mark.timeout(600)
def test_mvo_manager_books_through_dropin_match_reference(monkeypatch):
    """CPU (the reference's host QP runs here, not on the GPU box): each MVO manager's book
    from the drop-in compute_manager_weights (multi_manager.py:15-29 -> drop-in Simulation ->
    the reference's solver) equals the reference's."""
    import sys
    import types
    ref = "/root/reference"
    if not os.path.exists(os.path.join(ref, "portfolio_simulation.py")):
        pytest.skip("reference checkout not present")
    try:
        import cvxpy  # noqa: F401
    except ImportError:
        monkeypatch.setitem(sys.modules, "cvxpy", types.ModuleType("cvxpy"))
    monkeypatch.setenv("FMX_REFERENCE_DIR", ref)
    sys.dont_write_bytecode = True
    import factormodeling_amd._refload as RL
    import factormodeling_amd.multi_manager as MM
    import factormodeling_amd.portfolio_simulation as PS
    monkeypatch.setattr(RL, "_CACHE", {})
    factors_df, fw, settings = _mvo_frames(PS.SimulationSettings)
    for fac in NAMES_M:
        w, c = MM.compute_manager_weights(factors_df[fac].dropna(), settings, name=fac)
        gw, gc = _golden_book(fac)
        pd.testing.assert_series_equal(w, gw, check_names=False)
        np.testing.assert_array_equal(c[["long_count", "short_count"]].to_numpy(dtype=float), gc.to_numpy())
        assert list(c.index) == list(gc.index)


@pytest.mark.gpu
def test_compute_multimanager_weights_mvo_matches_reference(monkeypatch, caplog):
    """GPU: MVO managers' books (the reference's, per the CPU test above) folded by
    k_mm_combine equal the reference's combined weights and counts; the missing column 'zz'
    logs the reference's warning (multi_manager.py:42-44)."""
    import logging
    import factormodeling_amd.multi_manager as MM
    import factormodeling_amd.portfolio_simulation as PS
    books = {fac: _golden_book(fac) for fac in NAMES_M}
    monkeypatch.setattr(MM, "compute_manager_weights", lambda s, settings, name="manager": books[name])
    factors_df, fw, settings = _mvo_frames(PS.SimulationSettings)
    with caplog.at_level(logging.WARNING, logger="multi_manager"):
        w, counts = MM.compute_multimanager_weights(factors_df, fw, settings)
    assert any("Factor zz not in factors_df, skipping." in r.getMessage() for r in caplog.records)
    ref_idx = pd.MultiIndex.from_arrays([DATES_M[GM["w_d"]], SYMS_M[GM["w_s"]]], names=["date", "symbol"])
    pd.testing.assert_series_equal(w, pd.Series(GM["w_v"], index=ref_idx), check_exact=True)
    np.testing.assert_array_equal(counts.to_numpy(), GM["counts"])
