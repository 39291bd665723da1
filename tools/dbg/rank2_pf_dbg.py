"""Debug: persistent rank2 vs scipy rankdata on small / tied / many-row panels."""
import sys
import numpy as np
import torch
from scipy.stats import rankdata
sys.path.insert(0, ".")
import factormodeling_amd.engine as E


def check(A, D, tie, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((1, D, A))
    if tie == 1:
        X = np.round(X, 1)
    elif tie == 2:
        X = np.round(X * 3)
    got = E.cs_rank2(torch.as_tensor(X, device="cuda")).cpu().numpy().astype(np.int64)
    bad = []
    for d in range(D):
        exp = np.rint(2 * rankdata(X[0, d], method="average")).astype(np.int64)
        if not np.array_equal(got[0, d], exp):
            nb = int((got[0, d] != exp).sum())
            bad.append((d, nb))
    print(f"A={A} D={D} tie={tie}: bad rows {len(bad)} {bad[:5]}", flush=True)


for A in (8193, 10000):
    for tie in (0, 1, 2):
        for D in (4, 600):
            check(A, D, tie)
