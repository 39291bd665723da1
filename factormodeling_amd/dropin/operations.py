"""Drop-in ``operations`` module: put ``factormodeling_amd/dropin`` ahead of the reference
on ``sys.path`` and ``import operations`` resolves here."""
from factormodeling_amd.operations import *  # noqa: F401,F403
from factormodeling_amd.operations import __all__  # noqa: F401
