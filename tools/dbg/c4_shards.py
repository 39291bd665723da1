"""Debug: C4 step over N in-process shards vs one; where does the daily IC differ, and is it
the shard's own IC (local) or the gather?"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from factormodeling_amd import pipeline as PL  # noqa: E402
import factormodeling_amd.engine as E  # noqa: E402
from factormodeling_amd.comm import run_local_shards  # noqa: E402

D, A, F, world = (int(v) for v in sys.argv[1:5])
dev = torch.device("cuda", 0)
cfg = PL.workload_config("c4")
sp = PL.ShardedPanel(D, A, F, 0, 1, dev, seed=0, halo=cfg.halo)
col = {"_factors": [0]}
PL.run_step(sp, cfg, collect=col)
torch.cuda.synchronize()
d1 = col["daily"].cpu().numpy()
def rowsig(T):                                            # per-row signature: NaN count + nansum
    return torch.stack([torch.isnan(T).sum(-1).double(), torch.nan_to_num(T).sum(-1)], -1).cpu().numpy()


X1 = rowsig(sp.X)
R1 = rowsig(sp.R)
del sp, col
E._WORK.clear()
torch.cuda.empty_cache()


def shard(rank, comm):
    sp = PL.ShardedPanel(D, A, F, device=dev, seed=0, halo=cfg.halo, comm=comm)
    Xl0 = rowsig(sp.X[:, sp.halo:])                       # own rows before the step
    col = {"_factors": [0]}
    PL.run_step(sp, cfg, collect=col)
    torch.cuda.current_stream().synchronize()
    loc = E.ic_daily(sp.X, sp.R, (1,))[:, :, :, sp.halo:].cpu().numpy()   # this shard's own IC again
    torch.cuda.current_stream().synchronize()
    return (sp.d_lo, sp.d_hi, col["daily"].cpu().numpy(), loc, rowsig(sp.X), rowsig(sp.R), sp.halo, Xl0)


res = run_local_shards(world, shard)
for lo, hi, full, loc, X, R, h, Xl0 in res:
    eq = lambda a, b: (a == b) | (np.isnan(a) & np.isnan(b))  # noqa: E731
    badf = np.argwhere(~eq(full, d1))
    badl = np.argwhere(~eq(loc, d1[..., lo:hi]))
    xok = eq(X, X1[:, lo - h:hi]).all()
    rok = eq(R, R1[lo - h:hi]).all()
    x0ok = eq(Xl0, X1[:, lo:hi]).all()
    print(f"[{lo},{hi}) gathered-bad {len(badf)} first {badf[:2].tolist()} local-bad {len(badl)} "
          f"first {badl[:2].tolist()} X ok {xok} R ok {rok} X before step ok {x0ok}", flush=True)
