"""Time the daily trade list (method 'equal') on one C2-shaped signal panel.

    python tools/sim_bench.py [--dates 2520 --assets 5000 --reps 10 --cpu-dates 100]

GPU: k_trade_equal + ts delay on [D][A] fp64 resident in HBM, HIP events on the launch
stream.  CPU: the numpy oracle (oracle/simulation.py, test infrastructure: the checker,
timed here as a reported baseline) on the first --cpu-dates dates, scaled to D.  One JSON
line; units are asset-days/s.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import factormodeling_amd.engine as E  # noqa: E402
import oracle.simulation as OS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dates", type=int, default=2520)
    ap.add_argument("--assets", type=int, default=5000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--cpu-dates", type=int, default=100)
    ap.add_argument("--managers", type=int, default=20)
    a = ap.parse_args()
    D, A = a.dates, a.assets
    rng = np.random.default_rng(0)
    X = rng.standard_normal((D, A))
    X[rng.random(X.shape) < 0.01] = np.nan
    dev = torch.device("cuda", 0)
    Xd = torch.as_tensor(X, device=dev)
    W, c = E.trade_equal(Xd, 0.1)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(a.reps):
        W, c = E.trade_equal(Xd, 0.1)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    nd = min(a.cpu_dates, D)
    want, wc = OS.trade_equal(X[:nd], np.ones((nd, A), dtype=bool), 0.1)
    assert np.array_equal(W[:nd].cpu().numpy(), want, equal_nan=True)
    t0 = time.perf_counter()
    OS.trade_equal(X[:nd], np.ones((nd, A), dtype=bool), 0.1)
    cpu_s = (time.perf_counter() - t0) * D / nd
    # multi-manager: K ragged manager books (presence = non-NaN) + the weighted fold over
    # all D dates (multi_manager.py:32-81), device part only
    K = a.managers
    pres = torch.as_tensor((~np.isnan(X)).astype(np.uint8), device=dev)
    fw = np.random.default_rng(1).random((D, K))
    colmap, wdate = list(range(K)), np.arange(D)
    Wf = torch.empty((K, D, A), dtype=torch.float64, device=dev)
    cnt = torch.empty((K, D, 2), dtype=torch.float64, device=dev)

    def mm():
        for f in range(K):
            Wm, cm = E.trade_equal(Xd, 0.1, present=pres)
            Wf[f] = Wm
            cnt[f] = cm
        return E.mm_combine(Wf, cnt, fw, colmap, wdate)
    mm()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    mm()
    torch.cuda.synchronize()
    mm_ms = (time.perf_counter() - t0) * 1e3
    print(json.dumps({"workload": "trade_equal", "mm_managers": K, "mm_ms_wall": mm_ms, "dates": D, "assets": A, "gpu_ms": ms,
                      "gpu_asset_days_per_s": D * A / (ms / 1e3),
                      "alg_GBps": D * A * 24 / (ms * 1e6),  # dense: X in, Wraw out, shifted Wout out (one kernel)
                      "cpu_port_s_scaled": cpu_s, "cpu_asset_days_per_s": D * A / cpu_s, "cpu_dates_sampled": nd}))


if __name__ == "__main__":
    main()
