"""Probe: can two ranks of one process group share the box's single GPU over RCCL?

Spawns `world` ranks (env rendezvous on 127.0.0.1), each on cuda:0, and runs the three
collectives the sharded step uses (batch_isend_irecv ring, all_gather, int64 all_reduce).
usage: python tools/dbg/rccl_probe.py [world]"""
import os
import subprocess
import sys


def child():
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev)
    t = torch.full((4,), rank + 1, dtype=torch.int64, device=dev)
    dist.all_reduce(t)
    parts = [torch.empty(3, dtype=torch.float64, device=dev) for _ in range(world)]
    dist.all_gather(parts, torch.full((3,), float(rank), dtype=torch.float64, device=dev))
    s = torch.full((5,), float(rank), dtype=torch.float64, device=dev)
    r = torch.empty(5, dtype=torch.float64, device=dev)
    ops = []
    if rank + 1 < world:
        ops.append(dist.P2POp(dist.isend, s, rank + 1))
    if rank > 0:
        ops.append(dist.P2POp(dist.irecv, r, rank - 1))
    for q in (dist.batch_isend_irecv(ops) if ops else []):
        q.wait()
    torch.cuda.synchronize()
    print(f"rank {rank}: all_reduce {t.tolist()} gather {[p[0].item() for p in parts]} "
          f"recv {r[0].item() if rank else None}", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    if "RANK" in os.environ:
        child()
        sys.exit(0)
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK="0", WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT="29533")
        procs.append(subprocess.Popen([sys.executable, __file__], env=env))
    codes = [p.wait() for p in procs]
    print("exit codes", codes)
    sys.exit(max(abs(c) for c in codes))
