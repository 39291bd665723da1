"""The product never routes a hot-path function through the reference's code (VERDICT r3
item 10).  Only the host MVO solvers are delegated (``factormodeling_amd/_refload.py``);
these tests run the hot path with ``FMX_REFERENCE_DIR`` unset and the loader armed to fail.
"""
import importlib
import os
import sys

import numpy as np
import pandas as pd
import pytest

DROPIN = ["operations", "factor_selector", "factor_selection_methods", "composite_factor",
          "portfolio_simulation", "multi_manager"]


@pytest.fixture
def armed(monkeypatch):
    import factormodeling_amd._refload as RL
    monkeypatch.delenv("FMX_REFERENCE_DIR", raising=False)

    def boom(*a, **k):
        raise AssertionError("a hot-path call reached the reference loader")
    monkeypatch.setattr(RL, "load", boom)
    return RL


def test_dropin_imports_leave_reference_off_path(armed):
    for m in DROPIN:
        importlib.import_module("factormodeling_amd." + m)
    assert not any(os.path.isfile(os.path.join(p or ".", "factor_selection_methods.py")) and
                   os.path.abspath(p) != os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "factormodeling_amd",
                                                                      "dropin"))
                   for p in sys.path), "a reference checkout is on sys.path"
    assert not [k for k in sys.modules if k.startswith("_fmx_reference_")]


@pytest.mark.gpu
def test_hot_path_runs_without_reference(armed):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import factormodeling_amd.composite_factor as cf
    import factormodeling_amd.factor_selector as fs
    import factormodeling_amd.operations as ops
    rng = np.random.default_rng(3)
    D, A, F = 70, 30, 6
    dates = pd.bdate_range("2021-01-01", periods=D)
    syms = [f"S{i:02d}" for i in range(A)]
    idx = pd.MultiIndex.from_product([dates, syms], names=["date", "symbol"])
    names = [f"g{k // 3}_{k}_{['eq', 'flx', 'raw'][k % 3]}" for k in range(F)]
    df = pd.DataFrame(rng.standard_normal((D * A, F)), index=idx, columns=names)
    ret = pd.Series(0.01 * rng.standard_normal(D * A), index=idx, name="log_return")
    fret = pd.DataFrame(0.01 * rng.standard_normal((D, F)), index=pd.Index(dates, name="date"), columns=names)
    x = df[names[0]]
    for out in (ops.ts_mean(x, 20), ops.ts_decay(x, 150), ops.ts_rank(x, 60), ops.cs_rank(x), ops.cs_zscore(x),
                ops.cs_winsor(x), ops.market_neutralize(x)):
        assert len(out) == len(x)
    m = fs.single_factor_metrics(df, ret)
    assert len(m) == F
    sel = fs.FactorSelector(df, ret, fret, window=20, method="icir_top", method_kwargs={"top_x": 3}).prepare_selection()
    assert sel.shape[1] > 0
    assert len(cf.composite_factor_calculation(df, names[:4], method="zscore")) == len(df)
    assert len(cf.weighted_composite_factor(df, sel, method="rank")) == len(df)
    assert not [k for k in sys.modules if k.startswith("_fmx_reference_")]
