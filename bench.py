"""Benchmark: factor·asset·days/s of the device-resident ops + IC + selection pipeline.

    python bench.py --gpus N --steps K --warmup W [--dates D --assets A --factors F]

Default workload = BASELINE.json configs[1] (C2): 2,520 dates x 5,000 assets x 200
factors, synthetic data (SURVEY 8(d) generator, generated on the device).  A "step" is
one pass of factormodeling_amd.pipeline.run_step over the whole panel (9 operators, daily
IC/rank-IC/beta at lags 1-2, full-sample + rolling-window metrics, icir_top selection for
every processed day, fp64-MFMA factor Gram + greedy pruning).  For N > 1 the panel is
sharded by date (strong scaling: the same panel over N GPUs) with a halo exchange,
an IC all-gather and a Gram all-reduce over RCCL.

Rank 0 prints one JSON line (driver contract) with ``roofline`` (dominant kernel,
HIP-event timed inside the timed steps) and ``cpu_baseline`` (the numpy oracle port on
a bounded sample, 1 host core).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
FP64_PEAK_TFS = 78.6           # MI355X fp64 (vector = matrix) spec

# algorithmic bytes per factor·asset·day: a unary operator reads X once and
# writes once (16 B); the fused IC stage reads X once plus two R rows per (f, date) (8 + 16/F)
def bytes_per_unit(stage, F):
    kind = stage.split(":")[0]
    if kind in ("ts", "cs_rank", "cs", "winsor"):
        return 16.0
    if kind == "ts_set":            # X once + five outputs (mean, std, zscore, rank, decay)
        return 48.0
    if kind in ("cs_zscore_neutralize", "cs_rank_winsor"):   # X once + two outputs
        return 24.0
    if kind == "ic_daily":
        return 8.0 + 16.0 / F
    return None


# stage -> kernel-name prefix in the rocprofv3 PMC summary (profiles/traffic_c2.json)
STAGE_KERNEL = {"ic_daily": ("fmx::k_ic_daily_br<", "fmx::k_ic_daily_fr<"),
                "ts_set": "fmx::k_ts_set<", "cs_zscore_neutralize": "fmx::k_cs_moment_rg<0>",
                "cs_rank_winsor": "fmx::k_cs_rank_fa<",
                "cs_rank": ("fmx::k_cs_rank_br<", "fmx::k_cs_rank_fa<"),
                "winsor": "fmx::k_cs_quantile_br<0,", "cs:zscore": "fmx::k_cs_moment<0>",
                "cs:market_neutralize": "fmx::k_cs_moment<2>", "ts:mean": "fmx::k_ts_reg<1,",
                "ts:std": "fmx::k_ts_reg<2,", "ts:zscore": "fmx::k_ts_reg<4,", "ts:rank": "fmx::k_ts_reg<5,",
                "ts:decay": "fmx::k_ts_reg<6,"}
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic_c2.json")


def pmc_traffic(stage, dims):
    """HBM bytes per launch of the stage's kernel from the committed PMC summary (same
    panel dims only), else None."""
    try:
        t = json.load(open(TRAFFIC_FILE))
    except (OSError, ValueError):
        return None
    if list(t.get("dims", [])) != list(dims):
        return None
    key = ":".join(stage.split(":")[:2]).rstrip(":")
    pre = STAGE_KERNEL.get(key)
    for name, v in t.get("kernels", {}).items():
        if pre and name.startswith(pre if isinstance(pre, tuple) else (pre,)):
            return v["traffic_bytes"]
    return None


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--dates", type=int, default=2520)
    p.add_argument("--assets", type=int, default=5000)
    p.add_argument("--factors", type=int, default=200)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-sample-factors", type=int, default=1)
    p.add_argument("--stages", action="store_true", help="print per-stage times to stderr")
    p.add_argument("--selftest-dist", action="store_true",
                   help="CPU/gloo check of the rank launcher only (tests/test_bench_launch.py)")
    return p.parse_args()


def cpu_baseline(D, A, seed=0):
    """Time the numpy oracle port (test infrastructure; 1 core) on a bounded sample of the
    same workload: one factor over a 2520 x A slice for the operator set, plus daily IC
    over 120 dates.  Returns (factor·asset·days/s, description)."""
    import oracle.metrics as OM
    import oracle.ops as O
    rng = np.random.default_rng(seed)
    Ds = D
    x = rng.standard_normal((Ds, A))
    x[rng.random(x.shape) < 0.01] = np.nan
    r = 0.01 * rng.standard_normal((Ds, A))
    t0 = time.perf_counter()
    O.ts_mean(x, 20); O.ts_std(x, 20); O.ts_zscore(x, 20); O.ts_rank(x, 10); O.ts_decay(x, 20)
    O.cs_rank(x); O.cs_zscore(x); O.cs_winsor(x); O.market_neutralize(x)
    t_ops = time.perf_counter() - t0
    Di = min(Ds, 252)
    t0 = time.perf_counter()
    for t in range(2, Di):
        OM.daily_stats(x[t - 1], r[t])
        OM.daily_stats(x[t - 2], r[t])
    t_ic = (time.perf_counter() - t0) * (Ds / Di)
    units = Ds * A
    rate = units / (t_ops + t_ic)
    return rate, (f"numpy oracle (single thread), 1 factor x {Ds} dates x {A} assets: 9 operators "
                  f"({t_ops:.1f}s measured) + daily IC lags 1-2 ({t_ic:.1f}s, measured on {Di} dates, "
                  f"scaled to {Ds}); window metrics/selection/Gram not included")


def spawn_ranks(n):
    """``--gpus N`` without a torchrun launcher: start N ranks of this script as child
    processes (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set, one GPU each) before anything in
    this process touches the GPU, and exit with the worst child status."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    codes = [p.wait() for p in procs]
    bad = [c for c in codes if c != 0]
    return bad[0] if bad else 0


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.selftest_dist:
        rank = int(os.environ.get("RANK", "0"))
        if world > 1:
            dist.init_process_group("gloo")
            t = torch.tensor([float(rank + 1)])
            dist.all_reduce(t)
            world_seen = dist.get_world_size()
            dist.destroy_process_group()
        else:
            t, world_seen = torch.tensor([1.0]), 1
        if rank == 0:
            print(json.dumps({"n_gpus": world_seen, "rank_sum": float(t.item())}))
        return
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    from factormodeling_amd import pipeline as PL

    D, A, F = args.dates, args.assets, args.factors
    sp = PL.ShardedPanel(D, A, F, rank, world, dev, seed=0)
    cfg = PL.StepConfig()
    torch.cuda.synchronize()

    for _ in range(args.warmup):
        PL.run_step(sp, cfg)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    timers = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        PL.run_step(sp, cfg, timers=timers)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    stages = PL.stage_times(timers)
    ms_step = dt / args.steps * 1e3
    units = float(D) * A * F
    value = units / (dt / args.steps)

    # dominant kernel: the slowest HBM-priced stage (one launch of one kernel per step),
    # timed with HIP events recorded on the launch stream inside the timed steps
    op_stages = {k: v / args.steps for k, v in stages.items() if bytes_per_unit(k, F) is not None}
    dom, dom_ms = max(op_stages.items(), key=lambda kv: kv[1])
    local_units = float(F) * (sp.X.shape[1]) * A
    achieved = bytes_per_unit(dom, F) * local_units / (dom_ms * 1e-3) / 1e9
    # whole-step algorithmic bytes per unit of the HBM-priced stages (+ the Gram's X read)
    step_bpu = sum(bytes_per_unit(k, F) for k in op_stages) + 8.0
    traffic = pmc_traffic(dom, [sp.X.shape[1], A, F]) if world == 1 else None
    if args.stages and rank == 0:
        for k, v in sorted(stages.items(), key=lambda kv: -kv[1]):
            print(f"stage {k:28s} {v / args.steps:9.3f} ms", file=sys.stderr)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        rate, sample = cpu_baseline(D, A)
        cpu = {"value": rate, "unit": "factor·asset·days/s", "cores": 1, "kind": "port", "sample": sample}

    if rank == 0:
        line = {
            "metric": "factor·asset·days/s (ops+IC+select)",
            "value": value,
            "unit": "factor·asset·days/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SURVEY 8(d) generator, device-generated)",
            "config": {"workload": "C2 ops+IC+icir_top+corr-prune", "dates": D, "assets": A, "factors": F,
                       "parallelism": f"date-shard{world}", "sel_window": cfg.sel_window, "top_x": cfg.top_x},
            "roofline": {"kernel": dom, "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "algorithmic_bytes": bytes_per_unit(dom, F) * local_units, "ms": dom_ms},
            "stages_ms": {k: round(v / args.steps, 3) for k, v in stages.items()},
            "step_bytes_per_unit": step_bpu,
            "step_GBs": step_bpu * local_units / (ms_step * 1e-3) / 1e9,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
