"""Drop-in ``composite_factor`` module."""
from factormodeling_amd.composite_factor import (  # noqa: F401
    composite_factor_calculation, plot_factor_distributions, plot_quantile_backtests_log, weighted_composite_factor)
