"""Drop-in ``multi_manager`` module."""
import logging

from factormodeling_amd.multi_manager import (  # noqa: F401
    compute_manager_weights, compute_multimanager_weights, run_multimanager_backtest)

logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)-8s %(name)s %(message)s",
                    datefmt="%Y-%m-%d %H:%M:%S")
logger = logging.getLogger(__name__)
