"""engine.greedy_prune (blocked running-max walk) equals the direct walk "keep f iff
max |C[f, kept]| < rho" (np.max semantics: a NaN among the kept columns keeps f), for
symmetric and asymmetric C, NaN entries, every top_x cut and several thresholds."""
import numpy as np
import pytest

from factormodeling_amd.engine import greedy_prune


def walk(C, order, rho, top_x):
    kept = []
    for f in order:
        f = int(f)
        if kept and np.max(np.abs(C[f, kept])) >= rho:
            continue
        kept.append(f)
        if top_x is not None and len(kept) >= top_x:
            break
    return kept


@pytest.mark.parametrize("seed", range(12))
def test_greedy_prune_matches_walk(seed):
    rng = np.random.default_rng(seed)
    F = int(rng.integers(1, 300))
    B = rng.standard_normal((F, int(rng.integers(2, 30))))
    if seed % 4 == 0:
        B[rng.random(F) < 0.1] = 1.0                      # constant rows -> NaN correlations
    with np.errstate(invalid="ignore", divide="ignore"):
        C = np.atleast_2d(np.corrcoef(B)) if F > 1 else np.ones((1, 1))
    if seed % 3 == 1:
        C[rng.random(C.shape) < 0.03] = np.nan            # asymmetric NaNs
    order = rng.permutation(F)
    for rho in (0.2, 0.5, 0.7, 0.95):
        for top_x in (None, 1, 5, 70):
            assert greedy_prune(C, order, rho, top_x) == walk(C, order, rho, top_x)
