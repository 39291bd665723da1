"""C3 on the HIP path: the date-sharded step (BASELINE configs[2]) with the
product EngineBackend, its N shards run as N in-process threads on one MI355X
(factormodeling_amd.comm.LocalComm: halo send/recv, IC all-gather and the exact Gram
all-reduce are device copies ordered by HIP events), compared with the 1-shard HIP run of
the same panel; plus the exact Gram's split invariance on the device.

Tolerances: cross-sectional outputs, the daily IC series, window metrics, selections, the
correlation matrix C and the kept set are bit-identical at every shard count (C by the
exact fixed-point Gram, fmx_gram_exact); rolling outputs on owned dates restart their
Kahan/Welford state at the halo, so they agree to <= 1e-12 relative."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _one_shard(dev, D, A, F, cfg, seed):
    import torch
    from factormodeling_amd import pipeline as PL
    sp = PL.ShardedPanel(D, A, F, 0, 1, dev, seed=seed, halo=cfg.halo)
    col = {}
    w, kept = PL.run_step(sp, cfg, collect=col)
    torch.cuda.synchronize()
    return w.cpu().numpy(), kept, {k: (v.cpu().numpy() if hasattr(v, "cpu") else v) for k, v in col.items()}


@pytest.mark.timeout(400)
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_step_hip_matches_one_shard(dev, world):
    import torch
    from factormodeling_amd import pipeline as PL
    from factormodeling_amd.comm import run_local_shards
    D, A, F = 200, 700, 12
    cfg = PL.StepConfig(sel_window=60)
    w1, kept1, col1 = _one_shard(dev, D, A, F, cfg, 11)

    def shard(rank, comm):
        sp = PL.ShardedPanel(D, A, F, device=dev, seed=11, halo=cfg.halo, comm=comm)
        assert sp.halo == (cfg.halo if rank else 0)
        col = {}
        w, kept = PL.run_step(sp, cfg, collect=col)
        torch.cuda.current_stream().synchronize()
        return (sp.d_lo, sp.d_hi, w.cpu().numpy(), kept,
                {k: (v.cpu().numpy() if hasattr(v, "cpu") else v) for k, v in col.items()})

    res = run_local_shards(world, shard)
    assert [r[0] for r in res] == [PL.shard_bounds(D, world, r)[0] for r in range(world)]
    for lo, hi, w, kept, col in res:
        assert np.array_equal(w, w1), lo                              # selections
        assert kept == kept1, lo                                     # pruned set
        assert np.array_equal(col["C"], col1["C"]), lo               # exact Gram: same bits
        assert np.array_equal(col["daily"], col1["daily"], equal_nan=True), lo   # gathered IC series
        for k in ("summ", "win"):
            assert np.array_equal(col[k], col1[k], equal_nan=True), (lo, k)
        for kind, op, wn in cfg.ops:
            k = f"{kind}:{op or ''}:{wn or ''}"
            got, ref = col[k], col1[k][:, lo:hi]
            if kind == "ts":
                np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-13, equal_nan=True, err_msg=k)
            else:
                assert np.array_equal(got, ref, equal_nan=True), (lo, k)


@pytest.mark.timeout(200)
@pytest.mark.parametrize("F,A", [(12, 700), (200, 777), (37, 5000)])
def test_gram_exact_split_invariant_on_device(dev, F, A):
    """fmx_gram_exact over any split of the dates, limbs summed as integers, finalizes to
    the same G / N bits as one launch; and agrees with the oracle's Gram."""
    import torch
    import factormodeling_amd.engine as E
    import oracle.gram as OG
    rng = np.random.default_rng(F + A)
    D = 23
    X = rng.standard_normal((F, D, A))
    X[rng.random(X.shape) < 0.03] = np.nan
    X[0, 4] = 1.5                                   # constant row: sigma 0 -> invalid
    Xd = torch.as_tensor(X, device=dev)
    _, stats = E.cs_moment_stats("stats", Xd)
    L1, N1 = E.gram_exact(Xd, stats, 0, D)
    G1, Nf1 = E.gram_exact_finalize(L1, N1)
    for cuts in ([11], [1, 2, 17], [5, 6, 7, 8, 9, 22]):
        b = [0] + cuts + [D]
        L = torch.zeros_like(L1)
        N = torch.zeros_like(N1)
        for a0, a1 in zip(b[:-1], b[1:]):
            la, na = E.gram_exact(Xd, stats, a0, a1)
            L += la
            N += na
        G, Nf = E.gram_exact_finalize(L, N)
        assert torch.equal(G, G1) and torch.equal(Nf, Nf1), cuts
    Z, M = OG.zscore_exposures(X)
    Zf, Mf = Z.reshape(F, -1), M.reshape(F, -1)
    np.testing.assert_allclose(G1.cpu().numpy(), Zf @ Zf.T, rtol=1e-11, atol=1e-9)
    assert np.array_equal(Nf1.cpu().numpy(), Mf @ Mf.T)
    # accumulate=True adds into existing limbs
    L2, N2 = E.gram_exact(Xd, stats, 0, 11)
    E.gram_exact(Xd, stats, 11, D, limbs=L2, counts=N2, accumulate=True)
    G2, _ = E.gram_exact_finalize(L2, N2)
    assert torch.equal(G2, G1)
    # the z-score input path gives the same partials as the stats path (same z arithmetic)
    Zd = E.cs_moment("zscore", Xd)
    Lz, Nz = E.gram_exact(Zd, None, 0, D)
    Gz, Nzf = E.gram_exact_finalize(Lz, Nz)
    np.testing.assert_allclose(Gz.cpu().numpy(), G1.cpu().numpy(), rtol=1e-12, atol=1e-9)
    assert torch.equal(Nzf, Nf1)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("F,D,A,d0", [(40, 600, 300, 7), (260, 20, 5000, 0), (24, 40, 9000, 3), (30, 50, 5, 2)])
def test_gram_direct_exact_row_regimes(dev, F, D, A, d0):
    """The exact wide Gram across its row regimes: the z pass in 256-thread workgroups (<= 32
    numpy leaves; 600 dates = two z chunks of 32 date blocks, with a block phase), in
    512-thread ones (5000 assets), and rows it does not take (> 8192 or < 8 assets: the
    stats + z-while-staging path with its own stats) -- G and N vs the oracle."""
    import torch
    import factormodeling_amd.engine as E
    import oracle.gram as OG
    rng = np.random.default_rng(F * A + D)
    X = rng.standard_normal((F, D, A))
    X[rng.random(X.shape) < 0.05] = np.nan
    X[1, d0 + 1] = 0.25                              # constant row: invalid
    Xd = torch.as_tensor(X, device=dev)
    L, N = E.gram_direct_exact(Xd, d0, D, d_origin=0)
    G, Nf = E.gram_exact_finalize(L, N)
    Z, M = OG.zscore_exposures(X[:, d0:])
    Zf, Mf = Z.reshape(F, -1), M.reshape(F, -1)
    np.testing.assert_allclose(G.cpu().numpy(), Zf @ Zf.T, rtol=1e-11, atol=1e-9)
    assert np.array_equal(Nf.cpu().numpy(), Mf @ Mf.T)


@pytest.mark.parametrize("F,A", [(300, 257), (520, 1000)])
def test_gram_direct_exact_block_split_invariant(dev, F, A):
    """fmx_gram_direct_exact (the wide Gram): any split of the dates at
    absolute multiples of GRAM_DATE_BLOCK -- each piece a separate launch on its own local
    panel with its d_origin -- sums (as integers) to the same limbs / counts bits as one
    launch; G agrees with the float direct Gram and the oracle."""
    import torch
    import factormodeling_amd.engine as E
    import oracle.gram as OG
    rng = np.random.default_rng(F + A)
    D = 53
    X = rng.standard_normal((F, D, A))
    X[rng.random(X.shape) < 0.03] = np.nan
    X[1, 7] = 2.5                                   # constant row: invalid
    Xd = torch.as_tensor(X, device=dev)
    L1, N1 = E.gram_direct_exact(Xd)
    G1, Nf1 = E.gram_exact_finalize(L1, N1)
    B = E.GRAM_DATE_BLOCK
    for cuts in ([B], [B, 2 * B], [3 * B]):
        b = [0] + cuts + [D]
        L = torch.zeros_like(L1)
        N = torch.zeros_like(N1)
        for a0, a1 in zip(b[:-1], b[1:]):
            h = min(a0, 5)                          # a halo of preceding rows in the local panel
            loc = Xd[:, a0 - h:a1].contiguous()
            la, na = E.gram_direct_exact(loc, h, loc.shape[1], d_origin=a0 - h)
            L += la
            N += na
        G, Nf = E.gram_exact_finalize(L, N)
        assert torch.equal(G, G1) and torch.equal(Nf, Nf1), cuts
    Gf, Nff = E.gram_direct(Xd)
    np.testing.assert_allclose(G1.cpu().numpy(), Gf.cpu().numpy(), rtol=1e-12, atol=1e-9)
    assert torch.equal(Nf1, Nff)
    Z, M = OG.zscore_exposures(X)
    Zf, Mf = Z.reshape(F, -1), M.reshape(F, -1)
    np.testing.assert_allclose(G1.cpu().numpy(), Zf @ Zf.T, rtol=1e-11, atol=1e-9)
    assert np.array_equal(Nf1.cpu().numpy(), Mf @ Mf.T)


@pytest.mark.timeout(400)
@pytest.mark.parametrize("world", [2, 3])
def test_wide_gram_step_gpu_count_invariant(dev, world):
    """C4-shaped step (IC order + wide Gram + greedy prune) at F = 300 over LocalComm
    shards: C and the kept set are bit-identical to the 1-shard run (shards aligned to the
    Gram's date blocks, exact limbs all-reduced as int64)."""
    import torch
    from factormodeling_amd import pipeline as PL
    from factormodeling_amd.comm import run_local_shards
    D, A, F = 200, 300, 300
    cfg = PL.StepConfig(ops=[], ic_lags=(1,), select=False, gram=True, prune_top_x=None)
    _, kept1, col1 = _one_shard_nosel(dev, D, A, F, cfg, 5)

    def shard(rank, comm):
        sp = PL.ShardedPanel(D, A, F, device=dev, seed=5, halo=cfg.halo, comm=comm)
        assert sp.d_lo % PL.E.GRAM_DATE_BLOCK == 0
        col = {}
        _, kept = PL.run_step(sp, cfg, collect=col)
        torch.cuda.current_stream().synchronize()
        return kept, col["C"].cpu().numpy()

    for kept, C in run_local_shards(world, shard):
        assert np.array_equal(C, col1["C"])
        assert kept == kept1


def _one_shard_nosel(dev, D, A, F, cfg, seed):
    import torch
    from factormodeling_amd import pipeline as PL
    sp = PL.ShardedPanel(D, A, F, 0, 1, dev, seed=seed, halo=cfg.halo)
    col = {}
    w, kept = PL.run_step(sp, cfg, collect=col)
    torch.cuda.synchronize()
    return w, kept, {k: (v.cpu().numpy() if hasattr(v, "cpu") else v) for k, v in col.items()}


@pytest.mark.timeout(400)
@pytest.mark.parametrize("world", [2, 3])
def test_c5_sharded_step_selection_matches_one_shard(dev, world):
    """C5's IC, selection and composite run on the feature panel
    sign(ts_corr) * x / ts_std, whose rolling state restarts at each shard's halo, so the
    feature agrees with the 1-shard run to ~1e-15 relative, not bitwise.  The daily IC of the
    feature therefore agrees to <= 1e-12, and the discrete icir_top selection is checked to
    be identical on this panel (a selection can differ between GPU counts only where two
    factors' rolling rank ICIRs tie to within that noise)."""
    import torch
    from factormodeling_amd import pipeline as PL
    from factormodeling_amd.comm import run_local_shards
    D, A, F = 200, 700, 12
    cfg = PL.workload_config("c5")
    cfg.factor_chunk = 5
    w1, _, col1 = _one_shard(dev, D, A, F, cfg, 13)

    def shard(rank, comm):
        sp = PL.ShardedPanel(D, A, F, device=dev, seed=13, halo=cfg.halo, comm=comm)
        col = {}
        w, _ = PL.run_step(sp, cfg, collect=col)
        torch.cuda.current_stream().synchronize()
        return sp.d_lo, sp.d_hi, w.cpu().numpy(), col["daily"].cpu().numpy(), col["feature"].cpu().numpy()

    for lo, hi, w, daily, feat in run_local_shards(world, shard):
        np.testing.assert_allclose(feat, col1["feature"][:, lo:hi], rtol=1e-12, atol=1e-14, equal_nan=True)
        np.testing.assert_allclose(daily, col1["daily"], rtol=1e-12, atol=1e-14, equal_nan=True)
        assert np.array_equal(w, w1), lo


_BR_SCRIPT = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
from factormodeling_amd import pipeline as PL
from factormodeling_amd.comm import run_local_shards
dev = torch.device("cuda", 0)
D, A, F = 120, 700, 6
cfg = PL.StepConfig(sel_window=40)
sp = PL.ShardedPanel(D, A, F, 0, 1, dev, seed=5, halo=cfg.halo)
col1 = {}
w1, kept1 = PL.run_step(sp, cfg, collect=col1)
torch.cuda.synchronize()
def shard(rank, comm):
    s = PL.ShardedPanel(D, A, F, device=dev, seed=5, halo=cfg.halo, comm=comm)
    col = {}
    w, kept = PL.run_step(s, cfg, collect=col)
    torch.cuda.current_stream().synchronize()
    return w.cpu().numpy(), kept, col["daily"].cpu().numpy()
for w, kept, daily in run_local_shards(2, shard):
    assert np.array_equal(w, w1.cpu().numpy()) and kept == kept1
    assert np.array_equal(daily, col1["daily"].cpu().numpy(), equal_nan=True)
print("OK")
"""


@pytest.mark.timeout(300)
def test_sharded_step_under_br_rank_impl(dev):
    """with the splitter-bucket rank kernels (FMX_RANK_IMPL=br, read once per
    process: a child process) the fused date-range entry falls back to the two-pass form
    factor by factor instead of raising; the 2-shard step equals the 1-shard step."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, FMX_RANK_IMPL="br")
    r = subprocess.run([sys.executable, "-c", _BR_SCRIPT, root], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
