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
