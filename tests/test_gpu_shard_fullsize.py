"""C3 (BASELINE configs[2]) at the shard counts north_star names, at FULL size,
on one MI355X: the date-sharded step of C2 (2520 x 5000 x 200) as 4 and
8 in-process shards (factormodeling_amd.comm.LocalComm: every shard a thread on its own HIP
stream; halo slabs, the IC all-gather and the exact Gram all-reduce as device copies) and
C4 (2520 x 3000 x 2000) as 8 shards, compared with the 1-shard run of the same panel:
selections, kept sets and C bit-identical; sampled factors' operator outputs on owned
dates bit-identical (cross-sectional) or <= 1e-12 relative (rolling: the Kahan / Welford
state restarts at the halo).  RCCL itself needs one process per GPU: the driver's 8-GPU
run exercises it.  Each run frees its device memory before the next."""
import gc

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.fullsize]


@pytest.fixture
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    yield torch.device("cuda", 0)
    _free()


def _free():
    import torch
    import factormodeling_amd.engine as E
    E._WORK.clear()
    gc.collect()
    torch.cuda.empty_cache()


def _host(col, fs_keys):
    return {k: col[k].cpu().numpy() for k in fs_keys if k in col}


def _run(dev, world, D, A, F, cfg, fs):
    """(per-rank (d_lo, d_hi, w, kept, C, sampled ops on owned dates)) of a ``world``-shard
    step; world 1 runs without a comm."""
    import torch
    from factormodeling_amd import pipeline as PL
    from factormodeling_amd.comm import run_local_shards
    keys = [PL._op_key(*o) for o in cfg.ops]

    def shard(rank, comm):
        sp = PL.ShardedPanel(D, A, F, rank if comm is None else None, world if comm is None else None, dev,
                             seed=0, halo=cfg.halo, comm=comm)
        col = {"_factors": fs}
        w, kept = PL.run_step(sp, cfg, collect=col)
        torch.cuda.current_stream().synchronize()
        out = (sp.d_lo, sp.d_hi, None if w is None else w.cpu().numpy(), kept, col["C"].cpu().numpy(),
               _host(col, keys), col["daily"].cpu().numpy(), col["summ"].cpu().numpy())
        del sp, col, w
        return out

    res = [shard(0, None)] if world == 1 else run_local_shards(world, shard, timeout=900.0)
    _free()
    return res


def _compare(res1, res, cfg):
    (_, _, w1, kept1, C1, ops1, daily1, summ1), = res1
    for lo, hi, w, kept, C, ops, daily, summ in res:
        assert np.array_equal(C, C1), lo                            # exact Gram: same bits
        bad = np.argwhere(~((daily == daily1) | (np.isnan(daily) & np.isnan(daily1))))
        assert bad.size == 0, (lo, len(bad), bad[:8].tolist())      # gathered daily IC series
        assert np.array_equal(summ, summ1, equal_nan=True), lo      # full-sample metrics
        if w1 is not None:
            assert np.array_equal(w, w1), lo                        # selections
        assert kept == kept1, lo                                    # pruned set
        for k, v in ops.items():
            ref = ops1[k][:, lo:hi]
            if k.startswith("ts:"):
                np.testing.assert_allclose(v, ref, rtol=1e-12, atol=1e-13, equal_nan=True, err_msg=f"{k} @{lo}")
            else:
                assert np.array_equal(v, ref, equal_nan=True), (k, lo)


@pytest.mark.timeout(900)
def test_c2_full_step_4_and_8_shards_match_one(dev):
    from factormodeling_amd import pipeline as PL
    D, A, F = 2520, 5000, 200
    cfg = PL.workload_config("c2")
    fs = [3, 150]
    res1 = _run(dev, 1, D, A, F, cfg, fs)
    for world in (4, 8):
        res = _run(dev, world, D, A, F, cfg, fs)
        assert [r[0] for r in res] == [PL.shard_bounds(D, world, r)[0] for r in range(world)]
        _compare(res1, res, cfg)


@pytest.mark.timeout(900)
def test_c4_full_step_8_shards_match_one(dev, monkeypatch):
    from factormodeling_amd import pipeline as PL
    D, A, F = 2520, 3000, 2000
    cfg = PL.workload_config("c4")
    res1 = _run(dev, 1, D, A, F, cfg, [0])
    # eight shards' Gram workspaces on one device at once: smaller z chunks (the exact
    # block partials do not depend on the chunking)
    monkeypatch.setenv("FMX_GRAM_ZC_GB", "4")
    res = _run(dev, 8, D, A, F, cfg, [0])
    B = PL.E.GRAM_DATE_BLOCK
    assert all(r[0] % B == 0 for r in res)
    _compare(res1, res, cfg)
