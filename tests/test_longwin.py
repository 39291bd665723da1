"""Long rolling windows: the notebook's ts_decay sweep reaches 350 rows
(pipeline.ipynb:132,145) and hands off ts_decay(…, 80 / 150) (:268,310,510).

Fixtures: tests/golden/ops_longwin.npz (make_golden_longwin.py, the reference itself on a
420-date panel, dense and ragged).  CPU: the oracle against the fixtures.  GPU: the drop-in
operators (HIP kernels through libfmx) against the fixtures and the oracle.

Tolerances: bit-exact for ranks, rolling moments (pandas Kahan/Welford), shifts and
regressions.  ts_decay's reference is ``np.dot`` (OpenBLAS ddot, a host-CPU-dependent
summation order) over up to 350 terms, so it is pinned to a bound on that reordering:
|got - ref| <= 1e-13 * sum_k k|x_k| / sum_k k  (+1e-300), i.e. ~W ulps of the absolute
weighted sum -- a relative bound would be meaningless where the terms cancel.
ts_corr (builder-defined, pinned to pandas): |d| <= 1e-9 + 1e-6 |ref| (north_star 1e-6).
"""
import numpy as np
import pandas as pd
import pytest

import oracle.ops as O
from golden_io import assert_close, gather, load, series

FIX = "ops_longwin.npz"
DECAY_W = (80, 150, 175, 350)
RANK_W = (60, 200)
MOMENT_W = (175, 350)
LEAD = 200
TAGS = ("dense", "ragged")


def _panel(tag):
    z = load(FIX)
    st = {k.split("/", 1)[1]: v for k, v in z.items() if k.startswith(tag + "/")}
    D, A = len(st["dates"]), len(st["syms"])
    x = np.full((D, A), np.nan)
    y = np.full((D, A), np.nan)
    p = np.zeros((D, A), dtype=bool)
    x[st["in_x__d"], st["in_x__s"]] = st["in_x__v"]
    y[st["in_y__d"], st["in_y__s"]] = st["in_y__v"]
    p[st["in_x__d"], st["in_x__s"]] = True
    return st, x, y, (None if p.all() else p)


def _oracle_cases(x, y, p):
    cases = {}
    for w in DECAY_W:
        cases[f"ts_decay_{w}"] = (lambda w=w: O.ts_decay(x, w, p), "decay")
    for w in RANK_W:
        cases[f"ts_rank_{w}"] = (lambda w=w: O.ts_rank(x, w, p), "exact")
    for w in MOMENT_W:
        for op in ("sum", "mean", "std", "zscore", "diff", "delay"):
            cases[f"ts_{op}_{w}"] = (lambda w=w, op=op: getattr(O, "ts_" + op)(x, w, p), "exact")
    cases[f"ts_diff_m{LEAD}"] = (lambda: O.ts_diff(x, -LEAD, p), "exact")
    cases[f"ts_delay_m{LEAD}"] = (lambda: O.ts_delay(x, -LEAD, p), "exact")
    cases["ts_corr_175"] = (lambda: O.ts_corr(x, y, 175, p), "corr")
    return cases


def _decay_bound(x, w, p, ref_like):
    scale = O.ts_decay(np.abs(x), w, p)
    return 1e-13 * np.nan_to_num(scale, nan=0.0) + 1e-300


def _check(got, ref, kind, what, bound=None):
    if kind == "exact":
        assert_close(got, ref, exact=True, what=what)
    elif kind == "corr":
        assert_close(got, ref, rtol=1e-6, atol=1e-9, what=what)
    else:
        gn, rn = np.isnan(got), np.isnan(ref)
        assert np.array_equal(gn, rn), f"{what}: NaN mismatch"
        err = np.abs(got[~gn] - ref[~rn])
        assert (err <= bound[~gn]).all(), f"{what}: max err {err.max():.3e} over bound"
    # long windows must leave values to compare (not an all-NaN fixture)
    assert (~np.isnan(ref)).sum() > 0, what


@pytest.mark.parametrize("tag", TAGS)
def test_oracle_vs_reference_longwin(tag):
    st, x, y, p = _panel(tag)
    for key, (fn, kind) in _oracle_cases(x, y, p).items():
        out = fn()
        ref = st["out_" + key + "__v"]
        got = gather(out, st, "out_" + key)
        bound = None
        if kind == "decay":
            w = int(key.rsplit("_", 1)[1])
            bound = gather(_decay_bound(x, w, p, out), st, "out_" + key)
        _check(got, ref, kind, f"{tag}:{key}", bound)
    for rt in (0, 2):
        key = f"out_ts_regression_fast_175_1_{rt}"
        od, os_, ov = O.ts_regression_fast_long(st["in_x__d"], st["in_x__s"], st["in_y__v"], st["in_x__v"], 175, 1, rt)
        assert np.array_equal(od, st[key + "__d"]) and np.array_equal(os_, st[key + "__s"])
        assert_close(ov, st[key + "__v"], exact=True, what=f"{tag}:{key}")


@pytest.fixture(scope="module")
def ops():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import factormodeling_amd.operations as ops
    return ops


@pytest.mark.gpu
@pytest.mark.parametrize("tag", TAGS)
def test_gpu_longwin_vs_reference(ops, tag):
    st, x, y, p = _panel(tag)
    dates = pd.to_datetime(st["dates"])
    sx = series(st, "in_x", dates, name="fx")
    sy = series(st, "in_y", dates, name="fy")
    api = {}
    for w in DECAY_W:
        api[f"ts_decay_{w}"] = (lambda w=w: ops.ts_decay(sx, w), "decay")
    for w in RANK_W:
        api[f"ts_rank_{w}"] = (lambda w=w: ops.ts_rank(sx, w), "exact")
    for w in MOMENT_W:
        for op in ("sum", "mean", "std", "zscore", "diff", "delay"):
            api[f"ts_{op}_{w}"] = (lambda w=w, op=op: getattr(ops, "ts_" + op)(sx, w), "exact")
    api[f"ts_diff_m{LEAD}"] = (lambda: ops.ts_diff(sx, -LEAD), "exact")
    api[f"ts_delay_m{LEAD}"] = (lambda: ops.ts_delay(sx, -LEAD), "exact")
    api["ts_corr_175"] = (lambda: ops.ts_corr(sx, sy, 175), "corr")
    for key, (fn, kind) in api.items():
        got = fn()
        ref = st["out_" + key + "__v"]
        assert len(got) == len(ref), key
        bound = None
        if kind == "decay":
            w = int(key.rsplit("_", 1)[1])
            bound = gather(_decay_bound(x, w, p, None), st, "out_" + key)
        _check(got.to_numpy(dtype=np.float64), ref, kind, f"{tag}:{key}", bound)
    for rt in (0, 2):
        key = f"ts_regression_fast_175_1_{rt}"
        got = ops.ts_regression_fast(sy, sx, 175, lag=1, rettype=rt)
        assert len(got) == len(st["out_" + key + "__v"])
        assert_close(got.to_numpy(dtype=np.float64), st["out_" + key + "__v"], exact=True, what=f"{tag}:{key}")


@pytest.mark.gpu
@pytest.mark.parametrize("ragged", [False, True])
def test_gpu_decay_sweep_1_to_350(ops, ragged):
    """The notebook's sweep (pipeline.ipynb:132,145): every window 1…350 runs through the
    drop-in; each is checked against the oracle (ranks: bit-exact at a few windows)."""
    import factormodeling_amd.engine as E
    import torch
    rng = np.random.default_rng(11)
    D, A = 400, 96
    x = rng.standard_normal((D, A))
    x[rng.random((D, A)) < 0.002] = np.nan
    p = None
    if ragged:
        p = rng.random((D, A)) > 0.1
        p[:, 0] = True
    X = torch.as_tensor(x[None].copy(), device="cuda")
    P = None if p is None else torch.as_tensor(p.astype(np.uint8), device="cuda")
    for w in range(1, 351):
        got = E.ts("decay", X, w, present=P)[0].cpu().numpy()
        ref = O.ts_decay(x, w, p)
        gn, rn = np.isnan(got), np.isnan(ref)
        assert np.array_equal(gn, rn), w
        bound = _decay_bound(x, w, p, ref)
        assert (np.abs(got[~gn] - ref[~rn]) <= bound[~gn]).all(), w
    for w in (1, 2, 7, 33, 64, 129, 257, 350):
        got = E.ts("rank", X, w, present=P)[0].cpu().numpy()
        assert_close(got.ravel(), O.ts_rank(x, w, p).ravel(), exact=True, what=f"rank {w}")
