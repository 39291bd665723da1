"""Drop-in ``portfolio_simulation`` module."""
from factormodeling_amd.portfolio_simulation import Simulation, SimulationSettings  # noqa: F401
