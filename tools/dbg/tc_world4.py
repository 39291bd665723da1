"""Debug: the TorchComm (gloo, CUDA tensors) sharded step at world N on one GPU -- which
rank's halo / daily IC differ from the 1-process run.  usage: python tools/dbg/tc_world4.py [N]"""
import os
import socket
import sys

import numpy as np
import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
D, A, F = 200, 700, 12


def _rank(rank, world, port, q):
    import torch.distributed as dist
    from factormodeling_amd import pipeline as PL
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = PL.StepConfig(sel_window=60)
    sp = PL.ShardedPanel(D, A, F, rank, world, dev, seed=11, halo=cfg.halo)
    sp.exchange_halo()
    torch.cuda.synchronize()
    halo = (sp.X[:, :sp.halo].cpu().numpy(), sp.R[:sp.halo].cpu().numpy())
    sp2 = PL.ShardedPanel(D, A, F, rank, world, dev, seed=11, halo=cfg.halo)
    col = {}
    w, kept = PL.run_step(sp2, cfg, collect=col)
    torch.cuda.synchronize()
    q.put((rank, sp.d_lo, sp.d_hi, sp.halo, halo, col["daily"].cpu().numpy(), w.cpu().numpy()))
    dist.barrier()
    dist.destroy_process_group()


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    from factormodeling_amd import pipeline as PL
    cfg = PL.StepConfig(sel_window=60)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(60)
    sp = PL.ShardedPanel(D, A, F, 0, 1, torch.device("cuda", 0), seed=11, halo=cfg.halo)
    col = {}
    w1, _ = PL.run_step(sp, cfg, collect=col)
    X1, R1 = sp.X.cpu().numpy(), sp.R.cpu().numpy()
    d1 = col["daily"].cpu().numpy()
    for rank, lo, hi, h, (hx, hr), daily, w in res:
        if h:
            okx = np.array_equal(hx, X1[:, lo - h:lo], equal_nan=True)
            okr = np.array_equal(hr, R1[lo - h:lo], equal_nan=True)
        else:
            okx = okr = True
        dd = ~np.isclose(daily, d1, rtol=0, atol=0, equal_nan=True)
        bad_dates = sorted(set(np.nonzero(dd)[3].tolist()))
        print(f"rank {rank} [{lo},{hi}) halo {h}: halo X ok {okx} R ok {okr}; daily differs at "
              f"{len(bad_dates)} dates {bad_dates[:12]}; w equal {np.array_equal(w, w1.cpu().numpy())}", flush=True)


if __name__ == "__main__":
    main()
