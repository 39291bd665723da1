"""CPU oracle for the factor-panel hot path -- TEST INFRASTRUCTURE ONLY.

This package is a numpy restatement of the reference algorithms
(Yuming-Yang/FactorModeling: operations.py, factor_selector.py,
factor_selection_methods.py, composite_factor.py) on the dense panel layout
``x[D][A]`` (dates x assets, float64) with an optional presence mask.  Every
function cites the reference file:line it restates.

Who may import it: ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` -- and only as the checker / the timed CPU
baseline.  The product (``factormodeling_amd``) never imports it; a missing HIP
library makes the product raise instead of falling back here.

Pinning: the oracle is checked against golden vectors produced by running the
reference itself in the build container (``tests/golden/make_golden.py``;
``tests/test_oracle_golden.py``).  Builder-defined extensions with no reference
counterpart (``ts_corr``, corr-GEMM pruning) are marked "parity unpinned".
"""
from . import numerics, ops, metrics, composite, gram  # noqa: F401
