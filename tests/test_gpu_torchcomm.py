"""The date-sharded step through torch.distributed (comm.TorchComm) with the product HIP
backend: 2, 3 and 4 processes on the box's one MI355X over the gloo backend -- the same TorchComm
code path the driver's multi-GPU run drives over RCCL (RCCL itself refuses two ranks on one
device: DESIGN.md §7).  Selections, kept set, C and the gathered daily IC are bit-identical
to the 1-process run; rolling outputs on owned dates agree to 1e-12 (their Kahan / Welford
state restarts at the halo)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

D, A, F = 200, 700, 12


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    import traceback
    try:
        import torch
        import torch.distributed as dist
        from factormodeling_amd import pipeline as PL
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        cfg = PL.StepConfig(sel_window=60)
        sp = PL.ShardedPanel(D, A, F, rank, world, dev, seed=11, halo=cfg.halo)
        col = {}
        w, kept = PL.run_step(sp, cfg, collect=col)
        torch.cuda.synchronize()
        q.put((rank, sp.d_lo, sp.d_hi, w.cpu().numpy(), kept,
               {k: v.cpu().numpy() for k, v in col.items() if hasattr(v, "cpu")}))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        q.put(("error", rank, traceback.format_exc()))


@pytest.mark.timeout(500)
@pytest.mark.parametrize("world", [2, 3, 4])
def test_torchcomm_multi_process_step_matches_one_shard(world):
    """world 2: one boundary; world 3 and 4: middle ranks both receive and send their halo."""
    import torch
    import torch.multiprocessing as mp
    from factormodeling_amd import pipeline as PL
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = []
    try:
        for _ in range(world):
            r = q.get(timeout=400)
            assert r[0] != "error", r[2]
            res.append(r)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    cfg = PL.StepConfig(sel_window=60)
    sp = PL.ShardedPanel(D, A, F, 0, 1, torch.device("cuda", 0), seed=11, halo=cfg.halo)
    col1 = {}
    w1, kept1 = PL.run_step(sp, cfg, collect=col1)
    col1 = {k: v.cpu().numpy() for k, v in col1.items() if hasattr(v, "cpu")}
    w1 = w1.cpu().numpy()
    for rank, lo, hi, w, kept, col in sorted(res, key=lambda r: r[0]):
        assert np.array_equal(w, w1), rank
        assert kept == kept1, rank
        assert np.array_equal(col["C"], col1["C"]), rank
        assert np.array_equal(col["daily"], col1["daily"], equal_nan=True), rank
        for k, v in col.items():
            if ":" in k:                     # operator outputs on the owned dates
                np.testing.assert_allclose(v, col1[k][:, lo:hi], rtol=1e-12, atol=1e-12, equal_nan=True,
                                           err_msg=f"{k} rank {rank}")


@pytest.mark.timeout(400)
def test_bench_multi_rank_over_gloo():
    """bench.py's multi-rank path (its own rank launcher, barrier + max-over-ranks timing,
    one JSON line from rank 0) with 2 ranks on the one GPU over gloo
    (FMX_BENCH_DIST_BACKEND=gloo; the driver's multi-GPU run uses RCCL)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, FMX_BENCH_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup",
                          "1", "--dates", "504", "--factors", "20"], env=env, capture_output=True, text=True,
                         timeout=360)
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "date-shard2"
    assert line["value"] > 0 and line["unit"] == "factor·asset·days/s"
    assert line["value"] == pytest.approx(504 * 5000 * 20 / (line["ms_per_step"] * 1e-3), rel=1e-6)
