"""Drop-in ``factor_selection_methods`` module."""
from factormodeling_amd.factor_selection_methods import (  # noqa: F401
    corr_prune_selector, factor_momentum_selector, icir_top_selector, ledoit_wolf_shrinkage, mvo_selector)
