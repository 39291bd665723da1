"""Debug: the daily IC of date slices of the C4 panel (one stream, no shards) vs the IC of
the whole panel."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from factormodeling_amd import pipeline as PL  # noqa: E402
import factormodeling_amd.engine as E  # noqa: E402

D, A, F, world = (int(v) for v in sys.argv[1:5])
dev = torch.device("cuda", 0)
sp = PL.ShardedPanel(D, A, F, 0, 1, dev, seed=0, halo=1)
full = E.ic_daily(sp.X, sp.R, (1,))
torch.cuda.synchronize()
for r in range(world):
    lo, hi = PL.shard_bounds(D, world, r, 16)
    a = max(lo - 1, 0)
    Xl = sp.X[:, a:hi].contiguous()
    Rl = sp.R[a:hi].contiguous()
    loc = E.ic_daily(Xl, Rl, (1,))[..., lo - a:]
    torch.cuda.synchronize()
    ref = full[..., lo:hi]
    bad = (~((loc == ref) | (torch.isnan(loc) & torch.isnan(ref)))).nonzero()
    print(f"[{lo},{hi}) rows {F * (hi - a)} elems {F * (hi - a) * A} bad {bad.shape[0]} first {bad[:2].tolist()}",
          flush=True)
    del Xl, Rl, loc
import oracle.metrics as OM  # noqa: E402
for f, t in ((0, 100), (0, 424), (5, 700), (1999, 2000), (0, 303), (0, 305)):
    n, ic, ric, beta = OM.daily_stats(sp.X[f, t - 1].cpu().numpy(), sp.R[t].cpu().numpy())
    print("oracle", f, t, (n, ic, ric, beta), "full", full[0, :, f, t].cpu().numpy().tolist(), flush=True)
