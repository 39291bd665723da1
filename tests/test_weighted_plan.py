"""composite_factor.weighted_plan (the host plan of weighted_composite_factor) is
vectorised; this pins it to the direct per-row restatement of composite_factor.py:251-290
(groups by prefix in first-appearance order, group sums in column order, normalised or
equal weights, pooled suffix column lists) on random selections, including groups of 8+
members (numpy's pairwise sum), rows that are not panel dates and all-zero selections."""
import numpy as np
import pytest

from factormodeling_amd import engine
from factormodeling_amd.composite_factor import weighted_plan


def plan_loop(pdate, W, names):
    W = np.asarray(W, dtype=np.float64)
    J, F = W.shape
    suffix = np.array([engine.suffix_code(n) for n in names], dtype=np.int32)
    pref = [n.split("_", 1)[0] for n in names]
    sel = W > 0
    KMAX = int(max(1, sel.sum(axis=1).max() if J else 1))
    out = {k: np.zeros((J, KMAX), t) for k, t in (("col", np.int32), ("suf", np.int32), ("gw", np.float64))}
    out["grp"] = np.full((J, KMAX), -1, np.int32)
    ncol, ngrp, pd_out = np.zeros(J, np.int32), np.zeros(J, np.int32), np.full(J, -1, np.int32)
    soff, scol = [0], []
    for j in range(J):
        cs = np.flatnonzero(sel[j]) if pdate[j] >= 0 else np.zeros(0, np.int64)
        if cs.size:
            gid, members, gs = {}, [], []
            for c in cs:
                g = gid.setdefault(pref[c], len(gid))
                if g == len(members):
                    members.append([])
                members[g].append(c)
                gs.append(g)
            gsum = [W[j, m].sum() for m in members]
            tot = sum(gsum)
            gw = [x / tot for x in gsum] if tot > 0 else [1 / len(gsum)] * len(gsum)
            pd_out[j], ncol[j], ngrp[j] = pdate[j], cs.size, len(gw)
            out["col"][j, :cs.size] = cs
            out["suf"][j, :cs.size] = suffix[cs]
            out["grp"][j, :cs.size] = gs
            out["gw"][j, :len(gw)] = gw
        for sc in range(1, 5):
            scol.extend(int(c) for c in cs if suffix[c] == sc)
            soff.append(len(scol))
    out.update(pdate=pd_out, ncol=ncol, ngrp=ngrp, KMAX=KMAX, soff=np.asarray(soff, np.int32),
               scol=np.asarray(scol or [0], np.int32))
    return out


@pytest.mark.parametrize("seed", range(8))
def test_weighted_plan_matches_loop(seed):
    rng = np.random.default_rng(seed)
    suf = list(engine.SUFFIXES) + ["", "_q"]
    F, J = int(rng.integers(1, 60)), int(rng.integers(1, 80))
    names = ["%s_f%d%s" % (rng.choice(list("abcde")), i, rng.choice(suf)) for i in range(F)]
    p = 0.9 if seed % 3 == 0 else 0.3
    W = np.where(rng.random((J, F)) < p, rng.random((J, F)), 0.0)
    if seed == 5:
        W[:] = 0.0
    pdate = np.where(rng.random(J) < 0.8, np.arange(J), -1)
    ref, got = plan_loop(pdate, W, names), weighted_plan(pdate, W, names)
    assert set(ref) == set(got)
    for k in ref:
        a, b = np.asarray(ref[k]), np.asarray(got[k])
        assert a.dtype == b.dtype and a.shape == b.shape and np.array_equal(a, b), k
