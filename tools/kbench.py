"""Per-kernel timing harness (development tool, not the driver bench).

    python tools/kbench.py [--dates D --assets A --factors F] [--ops cs_rank,ic,...] [--reps N]

The panel is generated on the host with numpy (SURVEY 8(d) statistics: N(0,1), 1% NaN,
5% rounded to one decimal) for a small factor block and tiled along the factor axis on
the device, so no torch RNG kernels run (rocprofv3 --pmc passes stay clean).  Each op is
timed with HIP events on the current stream; GB/s uses the algorithmic 16 B per
factor·asset·day of a unary operator (8 B for the IC stage).
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if "--phases" in sys.argv:   # phase-timer build of libfmx (make -C factormodeling_amd/csrc prof)
    os.environ["FMX_LIB"] = os.path.join(ROOT, "factormodeling_amd", "libfmx_prof.so")
from factormodeling_amd import engine as E  # noqa: E402
from factormodeling_amd import _lib  # noqa: E402


def read_phases():
    import ctypes
    lib = _lib.load()
    out = {}
    for tu in ("cs", "hot", "q", "ic"):
        buf = (ctypes.c_ulonglong * 32)()
        getattr(lib, "fmx_debug_phase_" + tu)(buf)
        v = [int(x) for x in buf]
        if any(v):
            tot = sum(v)
            out[tu] = [round(x / tot, 3) for x in v if x] + [f"total {tot * 10 / 1e6:.1f} ms-WG"]
    return out


def panel(D, A, F, seed=0, block=8):
    rng = np.random.default_rng(seed)
    fb = min(F, block)
    x = rng.standard_normal((fb, D, A))
    u = rng.random((fb, D, A))
    x = np.where(u < 0.05, np.round(x, 1), x)
    x[u > 0.99] = np.nan
    r = 0.01 * rng.standard_normal((D, A))
    r[rng.random((D, A)) < float(os.environ.get("KB_R_NAN", "0.005"))] = np.nan
    Xb = torch.as_tensor(x, device="cuda")
    reps = (F + fb - 1) // fb
    X = Xb.repeat(reps, 1, 1)[:F].contiguous()
    return X, torch.as_tensor(r, device="cuda")


_SET = {}


def _set_outs(X):
    if not _SET:
        _SET.update({k: torch.empty_like(X) for k in E.TS_SET})
    return _SET


_RK = {}


def _rank2(X):
    """doubled ranks of X (made once, by the fused rank pass)."""
    if "rk" not in _RK:
        _RK["rk"] = torch.empty(X.shape, dtype=E.RANK2_DTYPE, device=X.device)
        E.cs_rank_winsor(X, 0.01, 0.99, rank2=_RK["rk"])
    return _RK["rk"]


_PR = {}


def _pres(X):
    """a ragged presence mask (10 % of rows absent), made once."""
    if "p" not in _PR:
        g = torch.Generator(device="cpu").manual_seed(5)
        _PR["p"] = (torch.rand(X.shape[1:], generator=g) > 0.1).to(torch.uint8).to(X.device)
    return _PR["p"]


OPS = {
    "ts_mean": (lambda X, R, Y: E.ts("mean", X, 20, out=Y), 16),
    "ts_std": (lambda X, R, Y: E.ts("std", X, 20, out=Y), 16),
    "ts_zscore": (lambda X, R, Y: E.ts("zscore", X, 20, out=Y), 16),
    "ts_rank": (lambda X, R, Y: E.ts("rank", X, 10, out=Y), 16),
    "ts_decay": (lambda X, R, Y: E.ts("decay", X, 20, out=Y), 16),
    # long windows (any W: k_ts_win tiles for rank / decay, k_ts_rl / k_ts_ptr for moments)
    "ts_decay80": (lambda X, R, Y: E.ts("decay", X, 80, out=Y), 16),
    "ts_decay150": (lambda X, R, Y: E.ts("decay", X, 150, out=Y), 16),
    "ts_decay350": (lambda X, R, Y: E.ts("decay", X, 350, out=Y), 16),
    "ts_rank60": (lambda X, R, Y: E.ts("rank", X, 60, out=Y), 16),
    "ts_rank200": (lambda X, R, Y: E.ts("rank", X, 200, out=Y), 16),
    "ts_mean175": (lambda X, R, Y: E.ts("mean", X, 175, out=Y), 16),
    "ts_mean20_rg": (lambda X, R, Y: E.ts("mean", X, 20, present=_pres(X), out=Y), 16),
    "ts_std175_rg": (lambda X, R, Y: E.ts("std", X, 175, present=_pres(X), out=Y), 16),
    "ts_decay150_rg": (lambda X, R, Y: E.ts("decay", X, 150, present=_pres(X), out=Y), 16),
    "ts_rank10_rg": (lambda X, R, Y: E.ts("rank", X, 10, present=_pres(X), out=Y), 16),
    "cs_rank": (lambda X, R, Y: E.cs_rank(X, out=Y), 16),
    "cs_zscore": (lambda X, R, Y: E.cs_moment("zscore", X, out=Y), 16),
    "market_neutralize": (lambda X, R, Y: E.cs_moment("market_neutralize", X, out=Y), 16),
    "winsor": (lambda X, R, Y: E.cs_quantile_op("winsor", X, 0.01, 0.99, out=Y), 16),
    "ic": (lambda X, R, Y: E.ic_daily(X, R, (1, 2)), 8),
    "ts_set": (lambda X, R, Y: E.ts_set(X, _set_outs(X), 20, 10), 48),
    "ts_set60_20": (lambda X, R, Y: E.ts_set(X, _set_outs(X), 60, 20), 48),
    "cs_zn": (lambda X, R, Y: E.cs_zscore_neutralize(X, Y, _set_outs(X)["mean"]), 24),
    "cs_rw": (lambda X, R, Y: E.cs_rank_winsor(X, 0.01, 0.99, Y, _set_outs(X)["mean"]), 24),
    "cs_rw_rk": (lambda X, R, Y: E.cs_rank_winsor(X, 0.01, 0.99, Y, _set_outs(X)["mean"], rank2=_rank2(X)), 26),
    "cs_rwzn_rk": (lambda X, R, Y: E.cs_rank_winsor_zn(X, 0.01, 0.99, Y, _set_outs(X)["mean"], _set_outs(X)["std"],
                                                      _set_outs(X)["zscore"], rank2=_rank2(X)), 42),
    "ic_ranked": (lambda X, R, Y: E.ic_daily(X, R, (1, 2), rank2=_rank2(X)), 10),
    "cs_rw_ic": (lambda X, R, Y: E.cs_rank_winsor_ic(X, R, (1, 2), 0.01, 0.99, Y, _set_outs(X)["mean"],
                                                     rank2=_RK.setdefault("rk", torch.empty(X.shape, dtype=E.RANK2_DTYPE,
                                                                                            device=X.device))), 24),
    "ts_corr60": (lambda X, R, Y: E.ts_corr(X, R, 60, out=Y), 16),
    "cvf60": (lambda X, R, Y: E.corr_vol_feature(X, Y, 60, out=_set_outs(X)["mean"]), 24),
    "corr_feat60": (lambda X, R, Y: E.corr_feature(X, R, 60, out=Y), 16),
    "rank2": (lambda X, R, Y: E.cs_rank2(X, _RK.setdefault("rk2", torch.empty(X.shape, dtype=E.RANK2_DTYPE,
                                                                              device=X.device))), 10),
    "gram": (lambda X, R, Y: E.corr_matrix(X), 8),
    # the C2 step's Gram: exact fixed-point partials from the cs_zscore output (Y after cs_zn)
    "gram_exact_z": (lambda X, R, Y: E.gram_exact(Y, None), 8),
    # the C4 step's Gram straight from the panel (row stats + validity bits + tiles + popcount)
    "gram_direct": (lambda X, R, Y: E.gram_direct(X), 8),
    # the C4 step's exact Gram (absolute 16-date blocks folded into fixed-point limbs)
    "gram_direct_exact": (lambda X, R, Y: E.gram_direct_exact(X), 8),
    "gram_unfused": (lambda X, R, Y: E.gram(*E.zscore_exposures(X)), 8),
    "cs_stats": (lambda X, R, Y: E.cs_moment_stats("stats", X), 8),
}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--dates", type=int, default=2520)
    p.add_argument("--assets", type=int, default=5000)
    p.add_argument("--factors", type=int, default=200)
    p.add_argument("--ops", default=",".join(OPS))
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--phases", action="store_true")
    a = p.parse_args()
    D, A, F = a.dates, a.assets, a.factors
    X, R = panel(D, A, F)
    Y = torch.empty_like(X)
    units = float(D) * A * F
    res = {}
    for name in a.ops.split(","):
        fn, bpu = OPS[name]
        fn(X, R, Y)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            fn(X, R, Y)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / a.reps
        res[name] = {"ms": round(ms, 3), "GBs": round(bpu * units / (ms * 1e-3) / 1e9, 1)}
        print(f"{name:18s} {ms:9.3f} ms  {res[name]['GBs']:8.1f} GB/s", flush=True)
        if a.phases:
            print("   phases:", read_phases(), flush=True)
    print(json.dumps({"dims": [D, A, F], "ops": res}))


if __name__ == "__main__":
    main()
