"""Golden vectors for ledoit_wolf_shrinkage (factor_selection_methods.py:60-117) made by
running the REFERENCE function in the build container (test infrastructure only):

    python tests/golden/make_golden_lw.py

Inputs are numpy arrays (time x factors): the reference indexes ``returns_centered[k]``
by row, which is row access only for an ndarray.  Cases: generic, a constant factor
(std 0: its pairs are left out of the mean correlation) and more factors than
observations.  (A single factor makes the reference raise ValueError in np.diag of the 0-d
np.cov; tests/test_selectors.py checks the same error.)  Writes ledoit_wolf.npz.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import OUT, import_reference  # noqa: E402


def cases():
    rng = np.random.default_rng(11)
    a = rng.standard_normal((60, 8)) * 0.02
    b = rng.standard_normal((40, 5)) * 0.01
    b[:, 2] = 0.003                               # constant factor
    d = rng.standard_normal((6, 9)) * 0.05        # p > n
    return {"generic": a, "const": b, "wide": d}


def main():
    _, _, ref_fsm, _ = import_reference()
    out = {}
    for name, x in cases().items():
        out[f"{name}_in"] = x
        out[f"{name}_out"] = np.asarray(ref_fsm.ledoit_wolf_shrinkage(x), dtype=np.float64)
    np.savez(os.path.join(OUT, "ledoit_wolf.npz"), **out)
    print("wrote", sorted(out))


if __name__ == "__main__":
    main()
