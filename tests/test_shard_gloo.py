"""Date-sharded multi-rank step on CPU (gloo, world_size 2) vs a single-rank run.

The product's distributed logic (factormodeling_amd.pipeline: halo exchange by
send/recv, IC all-gather, Gram all-reduce, redundant selection) runs unchanged; the
per-shard compute is the numpy oracle (test infrastructure) instead of libfmx, so this
runs without a GPU.  On the GPU box the same code runs over RCCL with libfmx."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle.gram as OG
import oracle.metrics as OM
import oracle.ops as O

D, A, F, W = 90, 48, 4, 20


class OracleBackend:
    """numpy oracle behind the pipeline's backend interface (tests only)."""

    def op(self, kind, op, w, X, out):
        x = X.numpy()
        for f in range(x.shape[0]):
            if kind == "ts":
                fn = {"mean": O.ts_mean, "std": O.ts_std, "zscore": O.ts_zscore, "rank": O.ts_rank,
                      "decay": O.ts_decay}[op]
                r = fn(x[f], w)
            elif kind == "cs_rank":
                r = O.cs_rank(x[f])
            elif kind == "cs":
                r = {"zscore": O.cs_zscore, "market_neutralize": O.market_neutralize}[op](x[f])
            else:
                r = O.cs_winsor(x[f])
            out[f] = torch.from_numpy(r)
        return out

    def ic_daily(self, X, R, lags):
        x, r = X.numpy(), R.numpy()
        Fn, Dn, _ = x.shape
        out = np.full((len(lags), 4, Fn, Dn), np.nan)
        out[:, 0] = 0
        for li, L in enumerate(lags):
            for f in range(Fn):
                for t in range(L, Dn):
                    out[li, :, f, t] = OM.daily_stats(x[f, t - L], r[t])
        return torch.from_numpy(out)

    def ic_window(self, daily, d0s, d1s):
        dl = daily.numpy()
        Fn = dl.shape[1]
        out = np.full((len(d0s), Fn, 8), np.nan)
        for j, (a, b) in enumerate(zip(d0s, d1s)):
            for f in range(Fn):
                sel = dl[0, f, a:b] >= 3
                ic, ric, be = dl[1, f, a:b][sel], dl[2, f, a:b][sel], dl[3, f, a:b][sel]
                out[j, f, :7] = OM.summarize(ic, ric, be)
                out[j, f, 5] = np.sum(~np.isnan(be))
        return torch.from_numpy(out)

    def select_icir_top(self, metrics, use_rank, thr, top_x):
        m = metrics.numpy()
        J, Fn, _ = m.shape
        w = np.zeros((J, Fn))
        order = np.zeros((J, Fn), np.int32)
        for j in range(J):
            o = OM.nargsort_desc(m[j, :, 3])
            order[j] = o
            w[j, o] = OM.icir_top(o, m[j], thr, top_x, use_rank)
        return torch.from_numpy(order), torch.from_numpy(w)

    def zscore_exposures(self, X):
        Z, M = OG.zscore_exposures(X.numpy())
        return torch.from_numpy(Z), torch.from_numpy(M)

    def gram(self, Z, M):
        Zf = Z.reshape(Z.shape[0], -1).double()
        Mf = M.reshape(M.shape[0], -1).double()
        return Zf @ Zf.T, Mf @ Mf.T

    @staticmethod
    def greedy_prune(C, order, rho, top_x):
        Cn = C.numpy() if isinstance(C, torch.Tensor) else C
        return OG.greedy_prune(Cn, order, rho, top_x)


def _run(rank, world, port, q):
    import traceback
    try:
        from factormodeling_amd import pipeline as PL
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        cfg = PL.StepConfig(sel_window=W)
        be = OracleBackend()
        sp = PL.ShardedPanel(D, A, F, rank, world, torch.device("cpu"), seed=3)
        col = {}
        w, kept = PL.run_step(sp, cfg, be=be, collect=col)
        ops = {k: v.numpy() for k, v in col.items() if ":" in k}
        q.put((rank, sp.d_lo, sp.d_hi, w.numpy(), kept, col["C"].numpy(), col["summ"].numpy(), ops))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        q.put(("error", rank, traceback.format_exc()))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(600)
def test_two_rank_step_matches_single_rank():
    from factormodeling_amd import pipeline as PL
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = []
    for _ in range(2):
        r = q.get(timeout=500)
        assert r[0] != "error", r[2]
        res.append(r)
    res.sort(key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-rank reference (no process group needed for world == 1)
    cfg = PL.StepConfig(sel_window=W)
    sp = PL.ShardedPanel(D, A, F, 0, 1, torch.device("cpu"), seed=3)
    col = {}
    w1, kept1 = PL.run_step(sp, cfg, be=OracleBackend(), collect=col)
    for rank, lo, hi, w, kept, C, summ, ops in res:
        assert np.array_equal(w, w1.numpy()), rank            # selections identical on every rank
        assert kept == kept1, rank
        np.testing.assert_allclose(C, col["C"].numpy(), rtol=1e-12, atol=1e-14)
        np.testing.assert_allclose(summ, col["summ"].numpy(), rtol=1e-12, atol=1e-14, equal_nan=True)
        for k, v in ops.items():                               # operators on owned dates (halo warm-up)
            ref = col[k].numpy()[:, lo:hi]
            np.testing.assert_allclose(v, ref, rtol=1e-12, atol=1e-12, equal_nan=True, err_msg=k)


def test_shard_bounds_cover_dates():
    from factormodeling_amd import pipeline as PL
    for world in (1, 2, 3, 4, 8):
        per = (2520 + world - 1) // world
        spans = [(min(2520, r * per), min(2520, (r + 1) * per)) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == 2520
        assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
    assert PL.HALO >= max(w for k, o, w in PL.OPS if w) - 1 + 2
