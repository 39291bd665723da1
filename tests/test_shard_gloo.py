"""Date-sharded multi-rank step on CPU (gloo, world_size 2, 3 and 4) vs a single-rank run.

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

from oracle_backend import OracleBackend

D, A, F, W = 90, 48, 4, 20


def _run(rank, world, port, q, skip_halo=False):
    import traceback
    try:
        from factormodeling_amd import pipeline as PL
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        cfg = PL.StepConfig(sel_window=W)
        be = OracleBackend()
        sp = PL.ShardedPanel(D, A, F, rank, world, torch.device("cpu"), seed=3)
        if skip_halo:
            sp.exchange_halo_start = lambda: None    # negative control: no exchange
            sp.exchange_halo_finish = lambda h: None
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


def _launch(world, skip_halo=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_run, args=(r, world, port, q, skip_halo)) for r in range(world)]
    for p in procs:
        p.start()
    res = []
    for _ in range(world):
        r = q.get(timeout=500)
        assert r[0] != "error", r[2]
        res.append(r)
    res.sort(key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 3, 4])
def test_sharded_step_matches_single_rank(world):
    """2 ranks: one boundary; 3 ranks: a middle rank both receives and sends its halo;
    4 ranks: two middle ranks (the halo slabs travel as one batch_isend_irecv group)."""
    from factormodeling_amd import pipeline as PL
    res = _launch(world)
    # single-rank reference (no process group needed for world == 1)
    cfg = PL.StepConfig(sel_window=W)
    sp = PL.ShardedPanel(D, A, F, 0, 1, torch.device("cpu"), seed=3)
    col = {}
    w1, kept1 = PL.run_step(sp, cfg, be=OracleBackend(), collect=col)
    for rank, lo, hi, w, kept, C, summ, ops in res:
        assert np.array_equal(w, w1.numpy()), rank            # selections identical on every rank
        assert kept == kept1, rank
        # the Gram is an exact integer fixed-point sum: the same bits at every rank count
        assert np.array_equal(C, col["C"].numpy()), rank
        np.testing.assert_allclose(summ, col["summ"].numpy(), rtol=1e-12, atol=1e-14, equal_nan=True)
        for k, v in ops.items():                               # operators on owned dates (halo warm-up)
            ref = col[k].numpy()[:, lo:hi]
            np.testing.assert_allclose(v, ref, rtol=1e-12, atol=1e-12, equal_nan=True, err_msg=k)


@pytest.mark.timeout(600)
def test_skipped_halo_exchange_is_detected():
    """Halo rows start as NaN, so a rank that skips the exchange produces NaN rolling
    outputs on its first owned dates (and a different selection input)."""
    from factormodeling_amd import pipeline as PL
    res = _launch(2, skip_halo=True)
    cfg = PL.StepConfig(sel_window=W)
    sp = PL.ShardedPanel(D, A, F, 0, 1, torch.device("cpu"), seed=3)
    col = {}
    PL.run_step(sp, cfg, be=OracleBackend(), collect=col)
    rank, lo, hi, w, kept, C, summ, ops = res[1]
    ref = col["ts:mean:20"].numpy()[:, lo:hi]
    got = ops["ts:mean:20"]
    assert np.isnan(got[:, :5]).all() and not np.isnan(ref[:, :5]).all()


def test_shard_bounds_cover_dates():
    from factormodeling_amd import pipeline as PL
    for world in (1, 2, 3, 4, 8):
        per = (2520 + world - 1) // world
        spans = [(min(2520, r * per), min(2520, (r + 1) * per)) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == 2520
        assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
    assert PL.HALO >= max(w for k, o, w in PL.OPS if w) - 1 + 2
    # wide-Gram alignment: every rank starts on an absolute multiple of the date block
    B = PL.E.GRAM_DATE_BLOCK
    assert PL.shard_align(300) == B and PL.shard_align(200) == 1
    for world in (1, 2, 3, 4, 8):
        spans = [PL.shard_bounds(2520, world, r, B) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == 2520
        assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
        assert all(lo % B == 0 for lo, _ in spans)
        PL.check_sharding(2520, world, 61, B)
    # short panels split whole blocks evenly -- 200 dates = 13 blocks of 16 over 8
    # ranks leave no rank empty (the old ceil(D / world) rounding gave rank 7 [200, 200))
    for D, world in ((200, 8), (100, 4), (33, 3), (2520, 7)):
        spans = [PL.shard_bounds(D, world, r, B) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == D
        assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
        assert all(hi > lo for lo, hi in spans) and all(lo % B == 0 for lo, _ in spans)
        PL.check_sharding(D, world, 1, B)
    # the larger shares go to the lower (halo-sending) ranks -- D = 121 over 2
    # ranks with a 61-date halo: rank 0 owns the 61 dates it sends
    assert PL.shard_bounds(121, 2, 0) == (0, 61) and PL.shard_bounds(121, 2, 1) == (61, 121)
    PL.check_sharding(121, 2, 61)
    for D, world in ((121, 2), (2520, 7), (203, 8), (33, 3)):
        n = [hi - lo for lo, hi in (PL.shard_bounds(D, world, r) for r in range(world))]
        assert n == sorted(n, reverse=True) and max(n) - min(n) <= 1, (D, world, n)


def test_rank_owning_fewer_dates_than_halo_is_rejected():
    """a sending rank with fewer owned dates than the halo would ship its own
    not-yet-received halo rows; the sharding is rejected up front."""
    from factormodeling_amd import pipeline as PL
    with pytest.raises(ValueError, match="owns"):
        PL.check_sharding(50, 3, 21)        # 17 dates per rank < halo 21
    with pytest.raises(ValueError, match="owns"):
        PL.check_sharding(5, 8, 1)          # ranks with no dates at all
    PL.check_sharding(90, 3, 21)
    PL.check_sharding(2520, 8, 61)


@pytest.mark.parametrize("world", [2, 3])
def test_local_comm_shards_match_gloo_semantics(world):
    """The in-process LocalComm (threads; the GPU test's transport) gives the same results
    as the 1-rank step, bit for bit on C and the selections (oracle backend, CPU)."""
    from factormodeling_amd import pipeline as PL
    from factormodeling_amd.comm import run_local_shards
    cfg = PL.StepConfig(sel_window=W)

    def shard(rank, comm):
        sp = PL.ShardedPanel(D, A, F, device=torch.device("cpu"), seed=3, comm=comm)
        col = {}
        w, kept = PL.run_step(sp, cfg, be=OracleBackend(), collect=col)
        return sp.d_lo, sp.d_hi, w.numpy(), kept, col["C"].numpy(), {k: v.numpy() for k, v in col.items() if ":" in k}

    res = run_local_shards(world, shard)
    sp = PL.ShardedPanel(D, A, F, 0, 1, torch.device("cpu"), seed=3)
    col = {}
    w1, kept1 = PL.run_step(sp, cfg, be=OracleBackend(), collect=col)
    for lo, hi, w, kept, C, ops in res:
        assert np.array_equal(w, w1.numpy()) and kept == kept1
        assert np.array_equal(C, col["C"].numpy())
        for k, v in ops.items():
            np.testing.assert_allclose(v, col[k].numpy()[:, lo:hi], rtol=1e-12, atol=1e-12, equal_nan=True, err_msg=k)


def test_feature_panel_step_never_reuses_the_ranks_of_x():
    """a step that ranks X in its operator set AND builds the C5 feature panel
    must not feed X's ranks (or X's fused IC records) to the IC of the feature panel."""
    import torch
    from factormodeling_amd import pipeline as PL

    calls = []

    class Be:
        ranked_ic_max_a = 1 << 30

        def cs_rank_winsor(self, X, outs, rank2=None):
            outs[0].zero_()
            outs[1].zero_()
            if rank2 is not None:
                rank2.zero_()

        def op(self, kind, op, w, X, out):
            out.copy_(X)

        def ts_corr_into(self, X, R, w, out):
            out.fill_(0.5)

        def corr_vol_feature(self, X, C, w, out):
            out.copy_(X * 2.0)

        def ic_daily(self, X, R, lags, rank2=None):
            calls.append((X.data_ptr(), rank2))
            return torch.zeros((len(lags), 4, X.shape[0], X.shape[1]), dtype=X.dtype)

        def ic_window(self, daily, d0, d1):
            return torch.zeros((len(d0), daily.shape[1], 8), dtype=daily.dtype)

    cfg = PL.StepConfig(ops=[("cs_rank", None, None), ("winsor", None, None)], ret_ops=[("corr_vol", 5)],
                        select=False, gram=False, ic_lags=(1,))
    sp = PL.ShardedPanel(30, 8, 3, 0, 1, torch.device("cpu"), seed=1, halo=cfg.halo)
    PL.run_step(sp, cfg, be=Be())
    assert len(calls) == 1
    ptr, rank2 = calls[0]
    assert ptr == sp.feature.data_ptr() and rank2 is None
