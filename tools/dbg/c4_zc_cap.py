"""Debug: does FMX_GRAM_ZC_GB (smaller z chunks) change anything but speed?  C4 shapes, one
shard: daily IC + C with the default cap vs a 4 GB cap."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from factormodeling_amd import pipeline as PL  # noqa: E402
import factormodeling_amd.engine as E  # noqa: E402

D = int(sys.argv[1]) if len(sys.argv) > 1 else 640
A, F = 3000, 2000
dev = torch.device("cuda", 0)
cfg = PL.workload_config("c4")
out = []
for cap in (None, "4"):
    if cap:
        os.environ["FMX_GRAM_ZC_GB"] = cap
    sp = PL.ShardedPanel(D, A, F, 0, 1, dev, seed=0, halo=cfg.halo)
    x0 = sp.X[:, ::97, ::31].clone()
    col = {"_factors": [0]}
    PL.run_step(sp, cfg, collect=col)
    torch.cuda.synchronize()
    out.append((col["daily"].cpu().numpy(), col["C"].cpu().numpy(), bool(torch.equal(x0, sp.X[:, ::97, ::31]))))
    del sp, col
    E._WORK.clear()
    torch.cuda.empty_cache()
(d0, c0, ok0), (d1, c1, ok1) = out
bad = np.argwhere(~((d0 == d1) | (np.isnan(d0) & np.isnan(d1))))
print("D", D, "X intact", ok0, ok1, "C equal", np.array_equal(c0, c1), "daily bad", len(bad), bad[:5].tolist())
