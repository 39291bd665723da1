"""Full-size checks of the benchmark configs on one MI355X (BASELINE
configs[1], [3], [4]): the shape-dependent planning (the wide Gram's date blocks, the rank
kernels' row tiling, the IC's chunking, C5's factor chunks) runs at the sizes it is timed
at, and sampled outputs are checked against the oracle / plain fp64 recomputation.

* C2 (2520 x 5000 x 200): the whole step; 4 sampled factors' nine operator outputs
  bit-exact (decay <= 1e-12 rel) vs the oracle, their daily IC (both lags) on sampled
  dates vs the oracle's scipy restatement (<= 1e-9), the selection of sampled days
  recomputed from the step's window metrics (bit-exact sets), 64 sampled C entries vs a
  plain fp64 recomputation (<= 1e-10), and the kept set vs a host greedy walk of C.
* C4 (2520 x 3000 x 2000): the wide exact Gram; C symmetric with a unit diagonal on valid
  rows, 64 sampled entries + their pair counts vs plain fp64 / integer recomputation.
* C5 (2520 x 10000 x 500): 2 sampled factors' feature panel sign(ts_corr) * x / ts_std
  bit-exact vs the oracle, and their daily IC on sampled dates.
* Discrete outputs vs the oracle alone: the icir_top selections of 3
  (C2) / 2 (C5) consecutive processed days from ALL factors' window metrics recomputed by
  the oracle (daily_stats on a host process pool, summarize, icir_top), C5's weighted
  composite on 3 sampled days, C2's C entries among every kept pair, 256+ sampled C4
  entries including the pairs among the first 16 kept factors.

Each test frees its device memory before the next (C5 alone uses ~250 GB of HBM).
"""
import gc

import numpy as np
import pytest

from golden_io import assert_close

pytestmark = [pytest.mark.gpu, pytest.mark.fullsize]


@pytest.fixture
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    yield torch.device("cuda", 0)
    import factormodeling_amd.engine as E
    E._WORK.clear()
    gc.collect()
    torch.cuda.empty_cache()


def _zgram(Xf, Xg):
    """Plain fp64 z-score Gram entry of two [D][A] device rows (ddof 0; NaN / sigma 0 ->
    invalid) and its pair count."""
    import torch

    def z(x):
        m = ~torch.isnan(x)
        n = m.sum(1, keepdim=True)
        mu = torch.where(m, x, 0.0).sum(1, keepdim=True) / n
        sd = torch.sqrt(torch.where(m, (x - mu) ** 2, 0.0).sum(1, keepdim=True) / n)
        ok = m & (sd > 0)
        return torch.where(ok, (x - mu) / sd, 0.0), ok
    zf, mf = z(Xf)
    zg, mg = z(Xg)
    return float((zf * zg).sum()), int((mf & mg).sum())


def _greedy(C, order, rho, top):
    """Keep f iff max |C[f, kept]| < rho (a NaN max keeps it, as np.max propagates NaN)."""
    kept = []
    for f in order:
        m = np.max(np.abs(C[f, kept])) if kept else -np.inf
        if not (m >= rho):
            kept.append(int(f))
            if top is not None and len(kept) >= top:
                break
    return kept


def _check_days_vs_oracle(P, R, cfg, proc, wn, win, rng, ndays, what):
    """``ndays`` consecutive processed days: every factor's lag-L daily statistics over the
    days' windows by the oracle (tests/oracle_pool.py: oracle.metrics.daily_stats of the
    panel P's rows on a process pool), summarized per window; the step's weights wn[j] must
    equal the oracle's icir_top selection bit for bit, and the step's window metrics win[j]
    the oracle's to 1e-9."""
    import oracle_pool
    W, L = cfg.sel_window, cfg.ic_lags[-1]
    j0 = int(rng.integers(0, len(proc) - ndays))
    t_lo, t_hi = int(proc[j0]) - W + 1, int(proc[j0 + ndays - 1])
    T = np.arange(t_lo, t_hi)
    Xs = P[:, T - L].cpu().numpy()                              # exposures of target dates T
    od = oracle_pool.daily_many(Xs, R[T])                       # [F][len(T)][4]
    del Xs
    for j in range(j0, j0 + ndays):
        vals, wf = oracle_pool.window_selection(od, t_lo, int(proc[j]), W, cfg.icir_threshold, cfg.top_x)
        assert_close(win[j][:, [0, 1, 2, 3, 4, 6]].ravel(), vals[:, [0, 1, 2, 3, 4, 6]].ravel(), rtol=1e-9,
                     atol=1e-12, what=f"{what} window metrics, all factors, day {proc[j]}")
        assert wf.sum() > 0 and np.array_equal(wf, wn[j]), f"{what} selection day {proc[j]} vs the oracle"


def _prune_order(summ):
    """The step's pruning order: rank_IC_IR descending, NaN last, ties by position."""
    return np.argsort(-np.nan_to_num(summ[0, :, 3], nan=-np.inf), kind="stable")


def _oracle_full_sample(P, R, L, fs):
    """Full-sample lag-L metrics of factors ``fs`` by the oracle alone:
    oracle.metrics.daily_stats of every target date t in [L, D) on the host pool, the n >= 3
    rows summarized (factor_selector.py:26-73) -> [len(fs)][7]."""
    import oracle.metrics as OM
    import oracle_pool
    D = R.shape[0]
    out = np.empty((len(fs), 7))
    for c0 in range(0, len(fs), 50):                            # 50 factors (10 GB at C2) at a time
        sub = list(fs[c0:c0 + 50])
        Xs = P[sub, :D - L].cpu().numpy()                       # exposures of target dates L..D-1
        od = oracle_pool.daily_many(Xs, R[L:])
        del Xs
        for k in range(len(sub)):
            ok = od[k, :, 0] >= 3
            out[c0 + k] = OM.summarize(od[k, ok, 1], od[k, ok, 2], od[k, ok, 3])
    return out


def _check_summ(summ, vals, fs, what):
    """The step's full-sample metrics of factors fs vs the oracle's (<= 1e-9)."""
    got = summ[0][fs][:, [0, 1, 2, 3, 4, 6]]
    assert_close(got.ravel(), vals[:, [0, 1, 2, 3, 4, 6]].ravel(), rtol=1e-9, atol=1e-12,
                 what=f"{what} full-sample metrics")


def _plain_corr(X, chunk=126):
    """C of every factor pair in plain fp64 on the device (oracle/gram.py's spec: per-date
    z-scores with ddof 0, NaN / sigma 0 -> invalid, C = sum ZZ' / sum MM'), summed over date
    chunks -- independent of the exact-limb Gram it checks."""
    import torch
    F, D, A = X.shape
    G = torch.zeros((F, F), dtype=torch.float64, device=X.device)
    N = torch.zeros_like(G)
    for d0 in range(0, D, chunk):
        x = X[:, d0:d0 + chunk]
        m = ~torch.isnan(x)
        n = m.sum(2, keepdim=True)
        mu = torch.where(m, x, 0.0).sum(2, keepdim=True) / n
        sd = torch.sqrt(torch.where(m, (x - mu) ** 2, 0.0).sum(2, keepdim=True) / n)
        ok = m & (sd > 0)
        z = torch.where(ok, (x - mu) / sd, 0.0).reshape(F, -1)
        mf = ok.to(torch.float64).reshape(F, -1)
        G += z @ z.T
        N += mf @ mf.T
        del x, m, z, mf, ok
    return torch.where(N > 0, G / N, torch.zeros_like(G)).cpu().numpy()


@pytest.mark.timeout(900)
def test_c2_full_step_sampled_vs_oracle(dev):
    import torch
    import oracle.metrics as OM
    import oracle.ops as O
    from factormodeling_amd import pipeline as PL
    D, A, F = 2520, 5000, 200
    cfg = PL.workload_config("c2")
    sp = PL.ShardedPanel(D, A, F, 0, 1, dev, seed=0, halo=cfg.halo)
    fs = [0, 57, 123, 199]
    col = {"_factors": fs}
    w, kept = PL.run_step(sp, cfg, collect=col)
    torch.cuda.synchronize()
    X = sp.X[fs].cpu().numpy()
    R = sp.R.cpu().numpy()
    ref = {"ts:mean:20": lambda x: O.ts_mean(x, 20), "ts:std:20": lambda x: O.ts_std(x, 20),
           "ts:zscore:20": lambda x: O.ts_zscore(x, 20), "ts:rank:10": lambda x: O.ts_rank(x, 10),
           "ts:decay:20": lambda x: O.ts_decay(x, 20), "cs_rank::": O.cs_rank, "cs:zscore:": O.cs_zscore,
           "winsor::": O.cs_winsor, "cs:market_neutralize:": O.market_neutralize}
    for i in range(len(fs)):
        for key, fn in ref.items():
            got = col[key][i].cpu().numpy()
            exp = fn(X[i])
            if key == "ts:decay:20":                          # <= ~W ulps of sum k|x| / sum k
                bound = 1e-13 * np.nan_to_num(O.ts_decay(np.abs(X[i]), 20), nan=0.0) + 1e-300
                ok = np.isnan(got) == np.isnan(exp)
                assert ok.all() and (np.abs(np.nan_to_num(got - exp)) <= bound).all(), f"{key} f{fs[i]}"
            else:
                assert_close(got.ravel(), exp.ravel(), exact=True, what=f"{key} f{fs[i]}")
    # daily IC of the sampled factors on sampled target dates (lags 1 and 2)
    daily = col["daily"].cpu().numpy()                       # [L][4][F][D]
    rng = np.random.default_rng(0)
    for li, L in enumerate(cfg.ic_lags):
        for t in sorted(rng.choice(np.arange(L, D), 60, replace=False)):
            for i, f in enumerate(fs):
                n, ic, ric, beta = OM.daily_stats(X[i, t - L], R[t])
                assert daily[li, 0, f, t] == n
                assert_close(daily[li, 1:, f, t], np.array([ic, ric, beta]), rtol=1e-9, atol=1e-12,
                             what=f"IC L{L} f{f} t{t}")
    # window metrics of sampled days vs the oracle's summaries of the step's daily IC series,
    # and each day's icir_top selection recomputed from the step's window metrics
    win = col["win"].cpu().numpy()                           # [J][F][8]
    W = cfg.sel_window
    proc = np.arange(W, D - 1)
    wn = w.cpu().numpy()
    dl = daily[len(cfg.ic_lags) - 1]
    for j in sorted(rng.choice(len(proc), 40, replace=False)):
        i = proc[j]
        for f in fs:
            s = np.asarray(OM.summarize(dl[1, f, i - W + 1:i], dl[2, f, i - W + 1:i], dl[3, f, i - W + 1:i]))
            # device columns: IC, IC_IR, rank_IC, rank_IC_IR, tstat, n_beta, pct_pos, n_days
            # (the p-value is finished on the host from tstat and n_beta)
            got = win[j, f, [0, 1, 2, 3, 4, 6]]
            assert_close(got, s[[0, 1, 2, 3, 4, 6]], rtol=1e-9, atol=1e-12, what=f"window metrics day {i} f{f}")
        order = OM.nargsort_desc(win[j, :, 3])
        wo = OM.icir_top(order, win[j], cfg.icir_threshold, cfg.top_x)
        wf = np.zeros(F)
        wf[order] = wo
        assert np.array_equal(wf, wn[j]), f"selection day {i}"
    # three consecutive processed days selected from ALL factors' window
    # metrics recomputed by the oracle alone (daily_stats of the raw panel rows, summarize,
    # icir_top), bit-for-bit equal to the step's weights
    _check_days_vs_oracle(sp.X, R, cfg, proc, wn, win, rng, ndays=3, what="C2")
    # correlation Gram: 64 sampled entries vs plain fp64, every pair among the kept factors
    # too; kept = host greedy walk of C
    C = col["C"].cpu().numpy()
    pairs = [(int(a), int(b)) for a, b in rng.integers(0, F, size=(64, 2))]
    pairs += [(a, b) for x, a in enumerate(kept) for b in kept[x + 1:]]
    for a, b in pairs:
        g, n = _zgram(sp.X[a], sp.X[b])
        assert n > 0
        np.testing.assert_allclose(C[a, b], g / n, rtol=1e-10, atol=1e-12, err_msg=f"C[{a},{b}]")
        assert C[a, b] == C[b, a]
    summ = col["summ"].cpu().numpy()
    assert kept == _greedy(C, _prune_order(summ), cfg.prune_rho, cfg.top_x)
    # the pruning order pinned to the oracle alone -- every factor's
    # full-sample lag-1 metrics recomputed from the raw panel (all 2519 target dates), the
    # order they give equal to the step's, and the kept set walked over the oracle's order
    L0 = cfg.ic_lags[0]
    vals = _oracle_full_sample(sp.X, R, L0, list(range(F)))
    _check_summ(summ, vals, list(range(F)), "C2")
    oorder = OM.nargsort_desc(vals[:, 3])
    assert np.array_equal(oorder, _prune_order(summ)), "C2 pruning order vs the oracle"
    assert kept == _greedy(C, oorder, cfg.prune_rho, cfg.top_x)
    del sp, col, w


@pytest.mark.timeout(900)
def test_c4_full_wide_gram(dev):
    import torch
    import oracle.metrics as OM
    from factormodeling_amd import pipeline as PL
    D, A, F = 2520, 3000, 2000
    cfg = PL.workload_config("c4")
    sp = PL.ShardedPanel(D, A, F, 0, 1, dev, seed=0, halo=cfg.halo)
    col = {"_factors": [0]}
    _, kept = PL.run_step(sp, cfg, collect=col)
    torch.cuda.synchronize()
    C = col["C"]
    assert torch.equal(C, C.T)
    d = torch.diagonal(C)
    assert float((d - 1.0).abs().max()) <= 1e-12
    rng = np.random.default_rng(4)
    Cn = C.cpu().numpy()
    pairs = [(int(a), int(b)) for a, b in rng.integers(0, F, size=(256, 2))]
    pairs += [(0, F - 1), (F - 1, F - 1), (255, 256), (1023, 1024)]     # tile / block edges
    pairs += [(a, b) for x, a in enumerate(kept[:16]) for b in kept[x + 1:16]]   # the first kept
    for a, b in pairs:
        g, n = _zgram(sp.X[a], sp.X[b])
        np.testing.assert_allclose(Cn[a, b], g / n, rtol=1e-10, atol=1e-12, err_msg=f"C[{a},{b}]")
    summ = col["summ"].cpu().numpy()
    dorder = _prune_order(summ)
    assert kept == _greedy(Cn, dorder, cfg.prune_rho, None)
    # the first 32 factors of the pruning order and 32 others, their
    # full-sample metrics by the oracle alone; their relative order under the oracle's values
    # equals the step's order restricted to them
    others = rng.choice(dorder[32:], 32, replace=False)
    fs = [int(f) for f in dorder[:32]] + [int(f) for f in others]
    vals = _oracle_full_sample(sp.X, sp.R.cpu().numpy(), cfg.ic_lags[0], fs)
    _check_summ(summ, vals, fs, "C4")
    sub = np.asarray(fs)[OM.nargsort_desc(vals[:, 3])]
    pos = np.empty(F, dtype=np.int64)
    pos[dorder] = np.arange(F)
    assert np.array_equal(sub, np.asarray(fs)[np.argsort(pos[fs], kind="stable")]), "C4 order vs the oracle"
    # the daily IC the pruning order comes from, on sampled (factor, date) pairs across the
    # whole panel (rows past 4.19M of a 1-D grid of 1024-thread rows once went unwritten)
    daily = col["daily"]
    R = sp.R.cpu().numpy()
    L = cfg.ic_lags[0]
    for f, t in zip(rng.integers(0, F, 24), rng.integers(L, D, 24)):
        f, t = int(f), int(t)
        n, ic, ric, beta = OM.daily_stats(sp.X[f, t - L].cpu().numpy(), R[t])
        got = daily[0, :, f, t].cpu().numpy()
        assert got[0] == n, (f, t)
        assert_close(got[1:], np.array([ic, ric, beta]), rtol=1e-9, atol=1e-12, what=f"C4 IC f{f} t{t}")
    del sp, col, C, daily


@pytest.mark.timeout(900)
def test_c2_correlated_zoo_prune_vs_oracle(dev):
    """a full-size C2 panel whose factors are correlated (each a random
    mix of 6 common factors plus noise, the SURVEY 8(d) NaN mask kept), pruned over the whole
    ordered zoo so that the walk rejects factors.  The kept set must equal the greedy walk of
    a plain fp64 C over the ORACLE's order (full-sample lag-1 rank_IC_IR of every factor from
    oracle.metrics.daily_stats); no walk decision may sit within 1e-9 of rho."""
    import dataclasses
    import torch
    import oracle.metrics as OM
    from factormodeling_amd import pipeline as PL
    D, A, F = 2520, 5000, 200
    cfg = dataclasses.replace(PL.workload_config("c2"), prune_top_x=None)
    sp = PL.ShardedPanel(D, A, F, 0, 1, dev, seed=3, halo=cfg.halo)
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    K = 6
    mix = torch.randn((F, K), generator=g, dtype=torch.float64, device=dev)
    for d0 in range(0, D, 252):                                # in place, 252 dates at a time
        base = torch.randn((K, min(252, D - d0), A), generator=g, dtype=torch.float64, device=dev)
        noise = torch.randn((F, base.shape[1], A), generator=g, dtype=torch.float64, device=dev)
        z = torch.einsum("fk,kda->fda", mix, base) + 0.6 * noise
        x = sp.X[:, d0:d0 + base.shape[1]]
        x.copy_(torch.where(torch.isnan(x), x, z))
        del base, noise, z
    col = {"_factors": [0]}
    _, kept = PL.run_step(sp, cfg, collect=col)
    torch.cuda.synchronize()
    summ = col["summ"].cpu().numpy()
    Cdev = col["C"].cpu().numpy()
    del col
    import factormodeling_amd.engine as E
    E._WORK.clear()
    gc.collect()
    torch.cuda.empty_cache()
    Cp = _plain_corr(sp.X)
    np.testing.assert_allclose(Cdev, Cp, rtol=1e-10, atol=1e-12)
    vals = _oracle_full_sample(sp.X, sp.R.cpu().numpy(), cfg.ic_lags[0], list(range(F)))
    _check_summ(summ, vals, list(range(F)), "C2 zoo")
    oorder = OM.nargsort_desc(vals[:, 3])
    assert np.array_equal(oorder, _prune_order(summ)), "C2 zoo pruning order vs the oracle"
    walk = _greedy(Cp, oorder, cfg.prune_rho, None)
    assert kept == walk
    assert 0 < len(walk) < F // 2, f"the zoo should be pruned hard ({len(walk)} kept)"
    for i, f in enumerate(oorder):                             # decisions clear of rho
        prior = [k for k in walk if list(oorder).index(k) < i]
        if prior:
            assert abs(np.max(np.abs(Cp[f, prior])) - cfg.prune_rho) > 1e-9, f
    del sp


@pytest.mark.timeout(900)
def test_c5_full_feature_sampled_vs_oracle(dev):
    import torch
    import oracle.metrics as OM
    import oracle.ops as O
    from factormodeling_amd import pipeline as PL
    D, A, F = 2520, 10000, 500
    cfg = PL.workload_config("c5")
    sp = PL.ShardedPanel(D, A, F, 0, 1, dev, seed=0, halo=cfg.halo)
    fs = [7, 431]
    col = {"_factors": fs}
    w, _ = PL.run_step(sp, cfg, collect=col)
    torch.cuda.synchronize()
    X = sp.X[fs].cpu().numpy()
    R = sp.R.cpu().numpy()
    feat = col["feature"].cpu().numpy()
    for i in range(len(fs)):
        exp = O.corr_vol_feature(X[i], R, 60)
        assert_close(feat[i].ravel(), exp.ravel(), exact=True, what=f"C5 feature f{fs[i]}")
    daily = col["daily"].cpu().numpy()
    rng = np.random.default_rng(5)
    for li, L in enumerate(cfg.ic_lags):
        for t in sorted(rng.choice(np.arange(60 + L, D), 20, replace=False)):
            for i, f in enumerate(fs):
                n, ic, ric, beta = OM.daily_stats(feat[i, t - L], R[t])
                assert daily[li, 0, f, t] == n
                assert_close(daily[li, 1:, f, t], np.array([ic, ric, beta]), rtol=1e-9, atol=1e-12,
                             what=f"C5 IC L{L} f{f} t{t}")
    assert w.shape == (D - cfg.sel_window - 1, F)
    # two consecutive days' selections from all 500 factors of the
    # feature panel by the oracle, and the weighted composite of 3 sampled days
    W = cfg.sel_window
    proc = np.arange(W, D - 1)
    wn = w.cpu().numpy()
    win = col["win"].cpu().numpy()
    _check_days_vs_oracle(sp.feature, R, cfg, proc, wn, win, rng, ndays=2, what="C5")
    import oracle.composite as OC
    comp = col["comp"]
    names = cfg.names or PL.factor_names(F)
    for j in sorted(rng.choice(len(proc), 3, replace=False)):
        d = int(proc[j])
        got = comp[d].cpu().numpy()
        exp = OC.weighted_composite_factor(sp.feature[:, d:d + 1].cpu().numpy(), names, [0], wn[j:j + 1],
                                           cfg.composite)[0]
        assert np.abs(got).sum() > 0
        assert_close(got, exp, rtol=1e-6, atol=1e-9, what=f"C5 weighted composite day {d}")
    del sp, col, w
