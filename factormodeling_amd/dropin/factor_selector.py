"""Drop-in ``factor_selector`` module.  Like the reference
(factor_selector.py:13-18) importing it configures INFO logging."""
import logging

logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)-8s %(name)s %(message)s",
                    datefmt="%Y-%m-%d %H:%M:%S")

from factormodeling_amd.factor_selector import (  # noqa: E402,F401
    FACTOR_SELECTION_METHODS, FactorSelector, single_factor_metrics)
from factormodeling_amd.factor_selection_methods import (  # noqa: E402,F401
    factor_momentum_selector, icir_top_selector, mvo_selector)
