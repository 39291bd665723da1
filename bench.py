"""Benchmark: factor·asset·days/s of the device-resident ops + IC + selection pipeline.

    python bench.py --gpus N --steps K --warmup W [--workload c2|c4|c5] [--dates D ...]

Default workload = BASELINE.json configs[1] (C2): 2,520 dates x 5,000 assets x 200
factors, synthetic data (SURVEY 8(d) generator, generated on the device).  A "step" is
one pass of factormodeling_amd.pipeline.run_step over the whole panel (9 operators, daily
IC/rank-IC/beta at lags 1-2, full-sample + rolling-window metrics, icir_top selection for
every processed day, fp64-MFMA factor Gram + greedy pruning).  For N > 1 the panel is
sharded by date (strong scaling: the same panel over N GPUs) with a halo exchange,
an IC all-gather and a Gram all-reduce over RCCL.

Other workloads (BASELINE configs[3], [4]; parity cases, not the driver's line):
  c4  2,520 x 3,000 x 2,000 factor zoo: daily IC + full-sample metrics for the pruning
      order, the 2,000 x 2,000 correlation Gram (fp64 MFMA, chunked by date) + greedy prune;
  c5  2,520 x 10,000 x 500: ts_corr(x, R, 60) over factor chunks feeding the feature panel
      sign(ts_corr) * x / ts_std(x, 60); its daily IC lags 1-2, 60-day window metrics,
      icir_top weights and the weighted composite (zscore) of the feature panel.

Rank 0 prints one JSON line (driver contract) with ``roofline`` (dominant kernel,
HIP-event timed inside the timed steps), ``cpu_baseline`` (the numpy oracle port on a
bounded sample, 16 host processes) and ``reference_cpu`` (the reference itself, timed in
the build container: SURVEY.md §6).
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
# writes once (16 B); the fused IC stage reads X once plus two R rows per (f, date) (8 + 16/F),
# plus the 4-B ranks when it starts from the operator set's ranks (which the rank pass writes)
def bytes_per_unit(stage, F, ranked=False):
    kind = stage.split(":")[0]
    if kind in ("ts", "cs_rank", "cs", "winsor"):
        return 16.0
    if kind == "ts_set":            # X once + five outputs (mean, std, zscore, rank, decay)
        return 48.0
    if kind == "cs_zscore_neutralize":  # X once + two outputs
        return 24.0
    if kind == "cs_rank_winsor":        # X once + two outputs + the doubled ranks (u16)
        return 26.0 if ranked else 24.0
    if kind == "cs_rank_winsor_zn":     # X once + four outputs + the doubled ranks (u16)
        return 42.0 if ranked else 40.0
    if kind == "cs_rank_winsor_ic":     # X once + two outputs + two R rows per (f, date); no ranks
        return 24.0 + 16.0 / F
    if kind == "rank_ic":               # ranks-only pass with the IC fused: X once + two R rows
        return 8.0 + 16.0 / F
    if kind == "rank2":              # ranks-only pass: X once + the u16 doubled ranks
        return 10.0
    if stage.startswith("ret:cvf"):     # C5 feature: X (+ the leaving value) and ts_corr in, F out
        return 24.0
    if stage.startswith("ret:corr_vol"):  # C5 fused ts_corr -> feature: X once + F out (R amortised)
        return 16.0
    if kind == "ret":                # ts_corr / ts_std vs returns: X once + out (R amortised)
        return 16.0
    if kind == "ic_daily":              # X once (+ its u16 ranks when ranked) + two R rows
        return (10.0 if ranked else 8.0) + 16.0 / F
    return None


# stage -> kernel-name prefix in the rocprofv3 PMC summaries (profiles/traffic_c*.json)
STAGE_KERNEL = {"ic_daily": ("fmx::k_ic_wave", "fmx::k_ic_daily_br<", "fmx::k_ic_daily_fr<"),
                "ts_set": "fmx::k_ts_set<", "rank2": ("fmx::k_cs_rank2_pf<", "fmx::k_cs_rank_fa<1024, 10, false, false", "fmx::k_cs_rank_fa<"),
                "ret:corr": ("fmx::k_ts_corr_fast<", "fmx::k_ts_corr_rl<"), "ret:corr_vol": "fmx::k_ts_corr_feat<", "ret:cvf": "fmx::k_ts_cvf_rl<", "gram": ("fmx::k_gram_zw<", "fmx::k_gram_f64w<", "fmx::k_gram_f64x<"),
                "cs_zscore_neutralize": "fmx::k_cs_moment_rg<0>",
                "cs_rank_winsor": "fmx::k_cs_rank_fa<", "cs_rank_winsor_ic": "fmx::k_cs_rank_fa<",
                "cs_rank_winsor_zn": "fmx::k_cs_rank_fa<512, 10, false, true, false, true",
                "rank_ic": "fmx::k_cs_rank_fa<",
                "cs_rank": ("fmx::k_cs_rank_br<", "fmx::k_cs_rank_fa<"),
                "winsor": "fmx::k_cs_quantile_br<0,", "cs:zscore": "fmx::k_cs_moment<0>",
                "cs:market_neutralize": "fmx::k_cs_moment<2>", "ts:mean": "fmx::k_ts_reg<1,",
                "ts:std": "fmx::k_ts_reg<2,", "ts:zscore": "fmx::k_ts_reg<4,", "ts:rank": "fmx::k_ts_reg<5,",
                "ts:decay": "fmx::k_ts_reg<6,"}
TRAFFIC_FILES = [os.path.join(ROOT, "profiles", f"traffic_{w}.json") for w in ("c2", "c4", "c5")]


def pmc_traffic(stage, dims):
    """HBM bytes per launch of the stage's kernel from the committed PMC summaries
    (tools/gpu_prof_r03.sh + tools/pmc_traffic.py): the summary of the same panel dims, or
    one of the same assets x factors on fewer dates (C4 / C5 are captured on 252 of the
    2520 dates: per-unit bytes x this launch's units), else None."""
    parts = stage.split(":")
    pre = STAGE_KERNEL.get(":".join(parts[:2]).rstrip(":")) or STAGE_KERNEL.get(parts[0])
    if not pre:
        return None
    pres = pre if isinstance(pre, tuple) else (pre,)
    for path in TRAFFIC_FILES:
        try:
            t = json.load(open(path))
        except (OSError, ValueError):
            continue
        td = list(t.get("dims", []))
        if td[1:] != list(dims)[1:]:
            continue
        ks = t.get("kernels", {})
        for p in pres:                       # the first prefix with a match wins
            for name in sorted(ks):
                if name.startswith(p):
                    v = ks[name]
                    return v["traffic_bytes"] if td == list(dims) else v["traffic_per_unit"] * float(
                        dims[0]) * dims[1] * dims[2]
    return None


# BASELINE.json configs: [1] C2, [3] C4, [4] C5 (D unspecified there: 2520)
WORKLOAD_DIMS = {"c2": (2520, 5000, 200), "c4": (2520, 3000, 2000), "c5": (2520, 10000, 500)}
WORKLOAD_NAME = {"c2": "C2 ops+IC+icir_top+corr-prune",
                 "c4": "C4 wide zoo: IC order + 2000x2000 corr Gram (fp64 MFMA) + greedy prune",
                 "c5": "C5 ts_corr/ts_std(60) feature -> its daily IC -> icir_top -> weighted composite"}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--workload", choices=["c2", "c4", "c5", "c1-dropin", "c2-dropin-slice"], default="c2")
    p.add_argument("--dates", type=int, default=None)
    p.add_argument("--assets", type=int, default=None)
    p.add_argument("--factors", type=int, default=None)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-workers", type=int, default=16, help="host processes of the CPU port baseline")
    p.add_argument("--stages", action="store_true", help="print per-stage times to stderr")
    p.add_argument("--selftest-dist", action="store_true",
                   help="CPU/gloo check of the rank launcher only (tests/test_bench_launch.py)")
    return p.parse_args()


def _port_worker(args):
    """One factor of the C2 step on the numpy oracle port (test infrastructure; a child
    process, no GPU): the 9 operators over all dates, daily IC lags 1-2 on a date sample
    (scaled), and the factor's exposures for the Gram.  Returns timings."""
    D, A, seed, ic_dates = args
    sys.path.insert(0, ROOT)
    import oracle.metrics as OM
    import oracle.numerics as nm
    import oracle.ops as O
    nm.FAST = True                 # 1-D pairwise sums by numpy's add.reduce (the same algorithm)
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((D, A))
    x = np.where(rng.random((D, A)) < 0.05, np.round(x, 1), x)
    x[rng.random(x.shape) < 0.01] = np.nan
    r = 0.01 * rng.standard_normal((D, A))
    t0 = time.perf_counter()
    O.ts_mean(x, 20); O.ts_std(x, 20); O.ts_zscore(x, 20); O.ts_rank(x, 10); O.ts_decay(x, 20)
    O.cs_rank(x); O.cs_zscore(x); O.cs_winsor(x); O.market_neutralize(x)
    t_ops = time.perf_counter() - t0
    Di = min(D, ic_dates)
    t0 = time.perf_counter()
    for t in range(2, Di):
        OM.daily_stats(x[t - 1], r[t])
        OM.daily_stats(x[t - 2], r[t])
    t_ic = (time.perf_counter() - t0) * (D / Di)
    return t_ops, t_ic


def cpu_baseline(D, A, workers=16, ic_dates=126):
    """The numpy oracle PORT of the C2 step on ``workers`` host processes (one factor each,
    all concurrent): operators + daily IC (sampled dates, scaled) per factor, then the
    window metrics + icir_top selection over all processed days and the factor Gram of the
    sampled factors.  Must run before this process touches the GPU (children are spawned).
    Returns (factor·asset·days/s, cores, description)."""
    import oracle.numerics as nm
    nm.FAST = True                 # numpy's own add.reduce for 1-D pairwise sums
    import concurrent.futures as cf
    import multiprocessing as mp
    import oracle.gram as OG
    import oracle.metrics as OM
    Fs = workers
    t0 = time.perf_counter()
    with _single_thread_children(), cf.ProcessPoolExecutor(max_workers=workers,
                                                           mp_context=mp.get_context("spawn")) as ex:
        res = list(ex.map(_port_worker, [(D, A, 1000 + f, ic_dates) for f in range(Fs)]))
    t_spawned = time.perf_counter() - t0
    # per-worker wall = ops + scaled IC; the concurrent run lasts as long as the slowest
    t_par = max(a + b for a, b in res)
    # window metrics (W = 60) + icir_top for every processed day over the sampled factors
    rng = np.random.default_rng(7)
    daily = rng.standard_normal((4, Fs, D)) * 0.05
    daily[0] = A
    t0 = time.perf_counter()
    W = 60
    for i in range(W, D - 1):
        vals = np.array([OM.summarize(daily[1, f, i - W + 1:i], daily[2, f, i - W + 1:i], daily[3, f, i - W + 1:i])
                         for f in range(Fs)])
        OM.icir_top(OM.nargsort_desc(vals[:, 3]), vals, -1.0, 5)
    t_sel = time.perf_counter() - t0
    # Gram of the sampled factors over a date sample (scaled)
    Dg = 63
    Xg = rng.standard_normal((Fs, Dg, A))
    t0 = time.perf_counter()
    OG.corr_matrix(Xg)
    t_gram = (time.perf_counter() - t0) * (D / Dg)
    wall = t_par + t_sel + t_gram
    units = float(Fs) * D * A
    desc = (f"numpy oracle port on {workers} host processes (one factor each, concurrent): {Fs} factors x {D} dates "
            f"x {A} assets; 9 operators + daily IC lags 1-2 ({ic_dates} dates measured, scaled) per factor "
            f"(slowest worker {t_par:.1f}s), window metrics + icir_top for {D - W - 1} days ({t_sel:.1f}s), "
            f"factor Gram ({Dg} dates measured, scaled: {t_gram:.1f}s); measured wall incl. process start "
            f"{t_spawned:.1f}s")
    return units / wall, workers, desc


class _single_thread_children:
    """Spawned port workers run single-threaded BLAS (one core each): without this every
    worker's numpy starts a full thread pool and 16 workers oversubscribe the host."""
    KEYS = ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.KEYS}
        for k in self.KEYS:
            os.environ[k] = "1"

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _port_worker_wide(args):
    """One factor of the C4 / C5 step on the numpy oracle port (child process, no GPU).
    c4: daily IC lag 1 on ``ic_dates`` dates (scaled to D).  c5: the feature
    sign(ts_corr(x, R, 60)) * x / ts_std(x, 60) over ``feat_dates`` dates (scaled), then its
    daily IC lags 1-2 on ``ic_dates`` dates (scaled).  Returns the factor's scaled seconds."""
    wl, D, A, seed, ic_dates, feat_dates = args
    sys.path.insert(0, ROOT)
    import oracle.metrics as OM
    import oracle.numerics as nm
    import oracle.ops as O
    nm.FAST = True                 # 1-D pairwise sums by numpy's add.reduce (the same algorithm)
    rng = np.random.default_rng(seed)
    Dm = min(D, max(ic_dates, feat_dates) + 2)
    x = rng.standard_normal((Dm, A))
    x = np.where(rng.random((Dm, A)) < 0.05, np.round(x, 1), x)
    x[rng.random(x.shape) < 0.01] = np.nan
    r = 0.01 * rng.standard_normal((Dm, A))
    t = 0.0
    lags = (1,)
    if wl == "c5":
        Df = min(Dm, feat_dates)
        t0 = time.perf_counter()
        x = O.corr_vol_feature(x[:Df], r[:Df], 60)
        t += (time.perf_counter() - t0) * (D / Df)
        x = np.where(np.isnan(x), rng.standard_normal(x.shape), x)    # past the warm-up: all-valid rows
        lags = (1, 2)
    Di = min(x.shape[0], ic_dates)
    t0 = time.perf_counter()
    for d in range(2, Di):
        for L in lags:
            OM.daily_stats(x[d - L], r[d])
    t += (time.perf_counter() - t0) * (D / (Di - 2))
    return t


def cpu_baseline_wide(wl, D, A, F, workers=16, ic_dates=64, feat_dates=504):
    """The numpy oracle PORT of the C4 / C5 step: per-factor work on
    ``workers`` host processes (one factor each, concurrent: the slowest worker's time x
    F / workers factors per worker), then the whole-zoo stages measured on samples and scaled
    -- C4: the full-sample metrics (summarize) of every factor, the 2000 x 2000 Gram (the
    z-score pass scaled by F·D·A, the Z^T Z product by F^2·D·A flops; numpy BLAS) and the
    greedy prune; C5: window metrics + icir_top for every processed day (scaled by F) and
    the weighted composite of every processed day (sampled days, scaled).  Must run before
    this process touches the GPU.  Returns (factor·asset·days/s, cores, description)."""
    import oracle.numerics as nm
    nm.FAST = True                 # numpy's own add.reduce for 1-D pairwise sums
    import concurrent.futures as cf
    import multiprocessing as mp
    import oracle.gram as OG
    import oracle.metrics as OM
    Fs = workers
    t0 = time.perf_counter()
    with _single_thread_children(), cf.ProcessPoolExecutor(max_workers=workers,
                                                           mp_context=mp.get_context("spawn")) as ex:
        res = list(ex.map(_port_worker_wide, [(wl, D, A, 1000 + f, ic_dates, feat_dates) for f in range(Fs)]))
    t_spawned = time.perf_counter() - t0
    t_par = max(res) * (F / workers)
    rng = np.random.default_rng(7)
    parts = [f"per-factor work on {workers} processes: slowest factor {max(res):.2f}s x {F}/{workers} "
             f"factors per process = {t_par:.1f}s"]
    if wl == "c4":
        daily = rng.standard_normal((4, Fs, D)) * 0.05
        t0 = time.perf_counter()
        for f in range(Fs):
            OM.summarize(daily[1, f], daily[2, f], daily[3, f])
        t_sum = (time.perf_counter() - t0) * (F / Fs)
        Fg, Dg = 256, 16
        Xg = rng.standard_normal((Fg, Dg, A))
        t0 = time.perf_counter()
        Z, M = OG.zscore_exposures(Xg)
        t_z = (time.perf_counter() - t0) * (F * D) / (Fg * Dg)
        Zf, Mf = Z.reshape(Fg, -1), M.reshape(Fg, -1)
        t0 = time.perf_counter()
        Zf @ Zf.T
        Mf @ Mf.T
        t_mm = (time.perf_counter() - t0) * (F / Fg) ** 2 * (D / Dg)
        Cg = np.corrcoef(rng.standard_normal((F, 64)))
        t0 = time.perf_counter()
        OG.greedy_prune(Cg, list(range(F)), 0.7, None)
        t_pr = time.perf_counter() - t0
        wall = t_par + t_sum + t_z + t_mm + t_pr
        parts.append(f"full-sample metrics {t_sum:.2f}s; Gram: z pass {t_z:.1f}s ({Fg}x{Dg}x{A} measured, scaled "
                     f"by F·D), Z^T Z + M^T M {t_mm:.1f}s ({Fg}x{Fg} over {Dg} dates measured, scaled by F^2·D); "
                     f"greedy prune {t_pr:.2f}s")
    else:
        W = 60
        daily = rng.standard_normal((4, Fs, D)) * 0.05
        t0 = time.perf_counter()
        J = D - W - 1
        Js = 200
        for i in range(W, W + Js):
            vals = np.array([OM.summarize(daily[1, f, i - W + 1:i], daily[2, f, i - W + 1:i],
                                          daily[3, f, i - W + 1:i]) for f in range(Fs)])
            OM.icir_top(OM.nargsort_desc(vals[:, 3]), vals, -1.0, 5)
        t_sel = (time.perf_counter() - t0) * (F / Fs) * (J / Js)
        import oracle.composite as OC
        from factormodeling_amd.pipeline import factor_names
        names = factor_names(F)
        nd = 8
        Xd = rng.standard_normal((F, nd, A))
        Wd = np.zeros((nd, F))
        for i in range(nd):
            Wd[i, rng.choice(F, 5, replace=False)] = 0.2
        t0 = time.perf_counter()
        OC.weighted_composite_factor(Xd, names, list(range(nd)), Wd, "zscore")
        t_comp = (time.perf_counter() - t0) * (J / nd)
        wall = t_par + t_sel + t_comp
        parts.append(f"window metrics + icir_top for {J} days ({Js} days x {Fs} factors measured, scaled: "
                     f"{t_sel:.1f}s); weighted composite ({nd} days measured, scaled: {t_comp:.1f}s)")
    units = float(F) * D * A
    desc = (f"numpy oracle port of {wl.upper()} ({F} factors x {D} dates x {A} assets): " + "; ".join(parts) +
            f"; per-factor samples: {ic_dates} IC dates" + (f", {feat_dates} feature dates" if wl == "c5" else "") +
            f"; measured wall incl. process start {t_spawned:.1f}s")
    return units / wall, workers, desc


# the reference itself (pandas/scipy as-is, 1 core) timed in the build
# container -- it cannot run on the GPU box (the reference never travels there).
REFERENCE_CPU = {
    "c1_measured": 3.25e4,
    "c2_extrapolated": 1.1e4,
    "unit": "factor·asset·days/s",
    "cores": 1,
    "source": "SURVEY.md §6: C1 (500x1000x20 ops+IC+select+composite) measured 307.4 s in the build container; "
              "C2 extrapolated from measured C2 slices: 8 operators ~3,200 s + winsor ~3,500 s + ts_decay ~6,100 s "
              "+ ts_rank ~159,000 s + single_factor_metrics ~1,700 s + FactorSelector ~57,500 s = ~2.3e5 s",
    "reconciliation": "BASELINE.md's 'about 4e4 f·a·d/s' (~17 h) sums the per-operator, single_factor_metrics and "
                      "FactorSelector extrapolations without ts_rank(10) (~44 h: pandas rolling.apply with a Python "
                      "callback per element) and the cs_winsor / ts_decay slices; the C2 operator set includes all "
                      "three, so the full extrapolation is ~2.3e5 s = 1.1e4 f·a·d/s",
}


def host_cpu():
    """(logical CPUs of this host, CPU model string) for the cpu_baseline record."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return os.cpu_count(), model


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


# the reference's own timings of the same calls (build container, 1 core)
DROPIN_REFERENCE_S = {
    "c1-dropin": {"cs_rank": 0.73, "cs_zscore": 0.52, "ts_mean(20)": 0.73, "ts_std(20)": 0.87,
                  "single_factor_metrics": 5.00, "FactorSelector(icir_top,60).prepare_selection": 292.2,
                  "weighted_composite_factor(zscore)": 7.34, "total": 307.4},
    # config-2 slices (2520 x 5000 x 2; single_factor_metrics measured at 200 dates, the
    # FactorSelector at 0.234 s per processed day): scaled to the slice's 2520 dates
    "c2-dropin-slice": {"cs_rank": 3.11, "cs_zscore": 2.94, "ts_mean(20)": 3.82, "ts_std(20)": 4.10,
                        "single_factor_metrics": 1.33 * 2520 / 200,
                        "FactorSelector(icir_top,60).prepare_selection": 0.234 * (2520 - 61)},
}


def dropin_bench(args):
    """The drop-in API end to end: the calls pipeline.ipynb makes
    (:216 single_factor_metrics, :351-361 FactorSelector(icir_top, window=60).prepare_selection,
    :461-463 weighted_composite_factor, plus the C1 operators) on pandas MultiIndex input, with
    the host <-> device boundary broken out (factormodeling_amd.profiling: pandas -> dense,
    H2D, D2H, dense -> pandas, host planning; the rest of each call's wall time is the device
    work -- launches and kernels -- and Python glue).  Not the driver's line."""
    import pandas as pd
    from factormodeling_amd import profiling
    from factormodeling_amd.dropin import composite_factor as cf
    from factormodeling_amd.dropin import factor_selector as fsel
    from factormodeling_amd.dropin import operations as ops
    D, A, F = (500, 1000, 20) if args.workload == "c1-dropin" else (2520, 5000, 2)
    D, A, F = args.dates or D, args.assets or A, args.factors or F
    rng = np.random.default_rng(0)
    names = [f"g{k // 4:03d}_{k:04d}_{['eq', 'flx', 'long', 'short', 'raw'][k % 5]}" for k in range(F)]
    X = rng.standard_normal((D, A, F))
    tie = rng.random(X.shape) < 0.05
    X[tie] = np.round(X[tie], 1)
    X[rng.random(X.shape) < 0.01] = np.nan
    r = 0.01 * rng.standard_normal((D, A))
    r[1:] += 0.002 * np.nan_to_num(X[:-1, :, 0])
    r[rng.random((D, A)) < 0.005] = np.nan
    dates = pd.bdate_range("2015-01-01", periods=D)
    idx = pd.MultiIndex.from_product([dates, [f"S{i:05d}" for i in range(A)]], names=["date", "symbol"])
    df = pd.DataFrame(X.reshape(D * A, F), index=idx, columns=names)
    ret = pd.Series(r.reshape(-1), index=idx, name="log_return")
    fret = pd.DataFrame(0.01 * rng.standard_normal((D, F)), index=pd.Index(dates, name="date"), columns=names)
    state = {}

    def sel_call():
        state["sel"] = fsel.FactorSelector(df, ret, fret, window=60, method="icir_top",
                                           method_kwargs={"top_x": 5, "icir_threshold": -1}).prepare_selection()
        return state["sel"]

    calls = [("cs_rank", lambda: ops.cs_rank(df)), ("cs_zscore", lambda: ops.cs_zscore(df)),
             ("ts_mean(20)", lambda: ops.ts_mean(df, 20)), ("ts_std(20)", lambda: ops.ts_std(df, 20)),
             ("single_factor_metrics", lambda: fsel.single_factor_metrics(df, ret)),
             ("FactorSelector(icir_top,60).prepare_selection", sel_call),
             ("weighted_composite_factor(zscore)", lambda: cf.weighted_composite_factor(df, state["sel"], "zscore"))]
    out = {}
    for name, fn in calls:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()                                   # cold: first call (index build, library / schedule setup)
        torch.cuda.synchronize()
        cold = time.perf_counter() - t0
        walls, phs = [], []
        for _ in range(max(1, args.steps)):
            with profiling.record() as ph:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                walls.append(time.perf_counter() - t0)
            phs.append(dict(ph))
        k = int(np.argsort(walls)[len(walls) // 2])
        wall, ph = walls[k], phs[k]
        rec = {"wall_s": wall, "cold_s": cold}
        rec.update({f"{p}_s": v for p, v in sorted(ph.items())})
        rec["device_and_glue_s"] = wall - sum(ph.values())
        ref = DROPIN_REFERENCE_S.get(args.workload, {}).get(name)
        if ref is not None:
            rec["reference_s"] = ref
            rec["speedup_vs_reference"] = ref / wall
        out[name] = rec
    tot = sum(v["wall_s"] for v in out.values())
    ref_tot = DROPIN_REFERENCE_S.get(args.workload, {}).get("total")
    line = {"metric": "drop-in API wall time (pandas in, pandas out)", "value": tot, "unit": "s",
            "higher_is_better": False, "n_gpus": 1, "steps": args.steps, "dtype": "f64",
            "data": "synthetic (SURVEY 8(d) generator, host numpy -> pandas MultiIndex)",
            "config": {"workload": args.workload, "dates": D, "assets": A, "factors": F},
            "calls": out, "reference_total_s": ref_tot,
            "speedup_vs_reference": (ref_tot / tot) if ref_tot else None,
            "reference_source": "SURVEY.md §6 (the reference itself, 1 core, build container)"}
    print(json.dumps(line))


def main():
    args = parse()
    if args.workload in ("c1-dropin", "c2-dropin-slice"):
        return dropin_bench(args)
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
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # before this process initialises the GPU: the port's workers are spawned children
        dims0 = WORKLOAD_DIMS[args.workload]
        Db, Ab, Fb = args.dates or dims0[0], args.assets or dims0[1], args.factors or dims0[2]
        if args.workload == "c2":
            rate, cores, sample = cpu_baseline(Db, Ab, args.cpu_workers)
        else:
            rate, cores, sample = cpu_baseline_wide(args.workload, Db, Ab, Fb, args.cpu_workers)
        ncpu, model = host_cpu()
        # cores: the worker processes the port actually used (one thread each); host_cpus:
        # the logical CPUs of the machine (the GPU box exposes many more than its CPU share)
        cpu = {"value": rate, "unit": "factor·asset·days/s", "cores": cores, "kind": "port", "sample": sample,
               "host_cpus": ncpu, "cpu_model": model}
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # one GPU per rank; FMX_BENCH_DIST_BACKEND=gloo (tests only) runs the same multi-rank
        # bench over gloo with the ranks sharing the visible devices (RCCL refuses two ranks
        # on one device)
        backend = os.environ.get("FMX_BENCH_DIST_BACKEND", "nccl")
        if backend != "nccl":
            local %= max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    from factormodeling_amd import pipeline as PL

    dims = WORKLOAD_DIMS[args.workload]
    D = args.dates or dims[0]
    A = args.assets or dims[1]
    F = args.factors or dims[2]
    cfg = PL.workload_config(args.workload)
    if os.environ.get("FMX_STEP_STREAMS") == "1":
        cfg.streams = True                      # A/B: the step's independent chains on 3 streams
    if os.environ.get("FMX_STEP_OVERLAP") == "1":
        cfg.overlap = True                      # A/B: the rolling set on a side stream
    sp = PL.ShardedPanel(D, A, F, rank, world, dev, seed=0, halo=cfg.halo)
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
    ranked = getattr(sp, "rank2", None) is not None   # the IC started from the rank pass's ranks
    bpu = lambda k: bytes_per_unit(k, F, ranked)      # noqa: E731
    op_stages = {k: v / args.steps for k, v in stages.items() if bpu(k) is not None}
    dom, dom_ms = max(op_stages.items(), key=lambda kv: kv[1])
    local_units = float(F) * (sp.X.shape[1]) * A
    achieved = bpu(dom) * local_units / (dom_ms * 1e-3) / 1e9
    # whole-step algorithmic bytes per unit of the HBM-priced stages (+ the Gram's X read)
    step_bpu = sum(bpu(k) for k in op_stages) + (8.0 if cfg.gram else 0.0)
    traffic = pmc_traffic(dom, [sp.X.shape[1], A, F]) if world == 1 else None
    roofline = {"kernel": dom, "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                "algorithmic_bytes": bpu(dom) * local_units, "ms": dom_ms}
    gram_ms = stages.get("gram", 0.0) / args.steps
    if cfg.gram and gram_ms > dom_ms:
        # the Gram dominates (C4): priced on MFMA -- the upper triangle incl. the diagonal of
        # G = Z^T Z, D*A*F*(F+1) flop (SURVEY 8(d) quotes the full square, 2*D*A*F^2)
        flops = float(sp.X.shape[1] - sp.halo) * A * F * (F + 1)
        tf = flops / (gram_ms * 1e-3) / 1e12
        gtraffic = pmc_traffic("gram", [sp.X.shape[1], A, F]) if world == 1 else None
        roofline = {"kernel": "gram", "bound": "mfma", "achieved": tf, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
                    "frac": tf / FP64_PEAK_TFS, "traffic": gtraffic, "algorithmic_flops": flops, "ms": gram_ms}
    if args.stages and rank == 0:
        for k, v in sorted(stages.items(), key=lambda kv: -kv[1]):
            print(f"stage {k:28s} {v / args.steps:9.3f} ms", file=sys.stderr)


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
            "config": {"workload": WORKLOAD_NAME[args.workload], "dates": D, "assets": A, "factors": F,
                       "parallelism": f"date-shard{world}", "sel_window": cfg.sel_window, "top_x": cfg.top_x,
                       "streams": 3 if (cfg.streams and cfg.ops) else 1},
            "roofline": roofline,
            "stages_ms": {k: round(v / args.steps, 3) for k, v in stages.items()},
            "step_bytes_per_unit": step_bpu,
            "step_GBs": step_bpu * local_units / (ms_step * 1e-3) / 1e9,
            "cpu_baseline": cpu,
            "reference_cpu": REFERENCE_CPU,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
