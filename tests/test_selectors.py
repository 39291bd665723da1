"""The drop-in host selectors (factor_selection_methods.py:6-58) against the reference's
pandas formulation, restated here as the spec: ``icir_top`` = nlargest over the
thresholded frame (ties in frame order), equal weights; ``momentum`` = positive window
return sums (NaN skipped), optionally capped, normalised.  Randomised frames with ties,
NaN metrics, NaN returns, top_x = 0 and all-negative windows; bit-exact weights, index and
name.  ``mvo_selector`` is the reference's own (loaded by path) and needs cvxpy: only its
missing-checkout error is checked here."""
import numpy as np
import pandas as pd
import pytest

import factormodeling_amd.factor_selection_methods as M


def _icir_spec(df, thr, top, use):
    col = "rank_IC_IR" if use else "IC_IR"
    sel = df[df[col] > thr].nlargest(top, col)
    vec = pd.Series(0.0, index=df.index, name="t")
    vec.loc[sel.index] = 1.0
    if vec.sum() > 0:
        vec = vec / vec.sum()
    return vec


def _momentum_spec(df, fr, mw):
    names = df.index.tolist()
    mom = fr.loc[:, names].sum().clip(lower=0)
    if mw < 1.0:
        mom = mom.clip(upper=mw)
    vec = pd.Series(0.0, index=mom.index, name="t")
    if mom.sum() > 0:
        vec = mom / mom.sum()
    return vec


@pytest.mark.parametrize("seed", range(4))
def test_icir_top_and_momentum_match_reference_formulation(seed):
    rng = np.random.default_rng(seed)
    for _ in range(60):
        F = int(rng.integers(1, 14))
        names = [f"f{i}" for i in range(F)]
        vals = rng.standard_normal((F, 2)) * 0.05
        vals = np.where(rng.random((F, 2)) < 0.25, np.round(vals, 2), vals)      # ties
        vals[rng.random((F, 2)) < 0.1] = np.nan
        df = pd.DataFrame(vals, index=names, columns=["IC_IR", "rank_IC_IR"])
        for use in (True, False):
            for top in (0, 1, 3, 5):
                got = M.icir_top_selector(df, None, None, None, "t", 0, icir_threshold=0.01, top_x=top,
                                          use_rank_icir=use)
                pd.testing.assert_series_equal(got, _icir_spec(df, 0.01, top, use), check_exact=True)
        W = int(rng.integers(1, 30))
        fr = pd.DataFrame(rng.standard_normal((W, F)) * 0.01 - (0.02 if rng.random() < 0.2 else 0.0),
                          columns=names)
        fr[fr.abs() < 0.002] = np.nan
        for mw in (1.0, 0.3, 0.005):
            got = M.factor_momentum_selector(df, None, None, fr, "t", 0, max_weight=mw)
            pd.testing.assert_series_equal(got, _momentum_spec(df, fr, mw), check_exact=True)


def test_mvo_selector_needs_the_reference_checkout(monkeypatch):
    monkeypatch.delenv("FMX_REFERENCE_DIR", raising=False)
    import factormodeling_amd._refload as RL
    monkeypatch.setattr(RL, "_CACHE", {})
    df = pd.DataFrame({"IC_IR": [0.1], "rank_IC_IR": [0.1]}, index=["a"])
    with pytest.raises(NotImplementedError, match="FMX_REFERENCE_DIR"):
        M.mvo_selector(df, None, None, pd.DataFrame({"a": [0.01]}), "t", 1)


def test_ledoit_wolf_shrinkage_matches_reference_golden():
    """factor_selection_methods.py:60-117 vs vectors the reference itself produced
    (tests/golden/make_golden_lw.py): generic, a constant factor (excluded from the mean
    correlation), more factors than observations -- bit for bit."""
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "ledoit_wolf.npz"))
    for name in ("generic", "const", "wide"):
        got = M.ledoit_wolf_shrinkage(g[f"{name}_in"])
        assert np.array_equal(got, g[f"{name}_out"]), name
    with pytest.raises(ValueError):                  # one factor: np.diag of a 0-d cov (as the reference)
        M.ledoit_wolf_shrinkage(np.zeros((10, 1)))
