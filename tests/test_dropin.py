"""The drop-in directory exposes the reference's module names and public symbols
(pipeline.ipynb:55-60 imports; factor_selector.py:20-24 registry) -- CPU only."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DROPIN = os.path.join(ROOT, "factormodeling_amd", "dropin")

REFERENCE_API = {
    "operations": ["ts_sum", "ts_mean", "ts_std", "ts_zscore", "ts_rank", "ts_diff", "ts_delay", "ts_decay",
                   "ts_backfill", "cs_rank", "cs_winsor", "cs_filter_center", "cs_zscore", "cs_bool", "cs_mean",
                   "sign", "power", "log", "abs_", "clip", "bucket", "group_mean", "group_neutralize",
                   "group_normalize", "group_rank_normalized", "market_neutralize", "ts_regression_fast",
                   "cs_regression"],
    "factor_selector": ["FACTOR_SELECTION_METHODS", "FactorSelector", "single_factor_metrics"],
    "factor_selection_methods": ["icir_top_selector", "factor_momentum_selector", "mvo_selector",
                                 "ledoit_wolf_shrinkage"],
    "composite_factor": ["composite_factor_calculation", "weighted_composite_factor", "plot_factor_distributions",
                         "plot_quantile_backtests_log"],
}


def test_dropin_modules_expose_reference_api():
    sys.path.insert(0, DROPIN)
    try:
        for mod, names in REFERENCE_API.items():
            sys.modules.pop(mod, None)
            m = importlib.import_module(mod)
            assert m.__file__.startswith(DROPIN), m.__file__
            missing = [n for n in names if not hasattr(m, n)]
            assert not missing, (mod, missing)
        fs = importlib.import_module("factor_selector")
        assert set(fs.FACTOR_SELECTION_METHODS) >= {"icir_top", "mvo", "momentum"}
    finally:
        sys.path.remove(DROPIN)
        for mod in REFERENCE_API:
            sys.modules.pop(mod, None)


def test_signatures_match_reference():
    import inspect
    import factormodeling_amd.composite_factor as cf
    import factormodeling_amd.factor_selector as fs
    import factormodeling_amd.operations as ops
    assert list(inspect.signature(ops.ts_regression_fast).parameters) == ["y", "x", "window", "lag", "rettype"]
    assert list(inspect.signature(ops.cs_rank).parameters) == ["series", "method"]
    assert list(inspect.signature(fs.FactorSelector.__init__).parameters) == [
        "self", "factors_df", "returns", "factor_ret_df", "window", "method", "method_kwargs"]
    assert list(inspect.signature(cf.weighted_composite_factor).parameters) == ["factors_df", "selection_df", "method"]


def test_no_gpu_means_loud_failure():
    """The product has no CPU fallback: without a HIP device every compute call raises."""
    import pytest
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import pandas as pd
    import factormodeling_amd.operations as ops
    from factormodeling_amd._lib import FmxError
    idx = pd.MultiIndex.from_product([pd.bdate_range("2020-01-01", periods=3), ["a", "b"]], names=["date", "symbol"])
    with pytest.raises(FmxError):
        ops.ts_mean(pd.Series(range(6), index=idx, dtype=float), 2)
