"""Device-resident factor-panel pipeline (one benchmark "step") and synthetic panels.

Step = the C2 hot path of BASELINE.json on a panel already resident in HBM:
  1. operator set per factor: ts_mean(20), ts_std(20), ts_zscore(20), ts_rank(10),
     ts_decay(20), cs_rank, cs_zscore, cs_winsor, market_neutralize
     (operations.py; each writes its own output panel)
  2. daily IC / rank-IC / beta at lag 1 (single_factor_metrics) and lag 2
     (FactorSelector windows) -- one launch; when the operator set ranks X (cs_rank), the
     IC starts from those ranks (fmx_ic_daily_ranked) instead of ranking X again
  3. full-sample metrics + rolling W-window metrics for every processed day
  4. icir_top selection per day (top_x=5, threshold=-1, factor_selector.py:94-139)
  5. correlation-based pruning: fp64-MFMA factor Gram + greedy prune (builder-defined)

Multi-GPU: ``ShardedPanel`` holds a rank's date shard plus a halo of the preceding
dates; ``run_step`` exchanges the halo, runs 1-2 on local dates, all-gathers the daily
IC series, runs 3-4 redundantly, all-reduces the Gram partials and prunes.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import contextlib
import os

import numpy as np
import torch

from . import engine as E

OPS = [("ts", "mean", 20), ("ts", "std", 20), ("ts", "zscore", 20), ("ts", "rank", 10), ("ts", "decay", 20),
       ("cs_rank", None, None), ("cs", "zscore", None), ("winsor", None, None), ("cs", "market_neutralize", None)]
MAX_LOOKBACK = 20          # longest rolling window in OPS
SEL_WINDOW = 60            # FactorSelector window (pipeline.ipynb:355)
HALO = MAX_LOOKBACK - 1 + 2  # rolling warm-up + IC lag 2


@dataclass
class StepConfig:
    """One benchmark step.  Defaults = C2 (BASELINE configs[1]); ``workload_config`` gives
    C4 (wide factor zoo: IC order + chunked 2000 x 2000 Gram + greedy prune) and C5
    (ts_corr / ts_std at 60 days over factor chunks, rolling-IC icir_top weights, weighted
    composite)."""
    sel_window: int = SEL_WINDOW
    top_x: int = 5
    icir_threshold: float = -1.0
    prune_rho: float = 0.7
    ops: list = field(default_factory=lambda: list(OPS))
    fuse: bool = True          # multi-output kernels: one read of X for several operators
    ic_lags: tuple = (1, 2)
    select: bool = True        # rolling-window metrics + icir_top per processed day
    gram: bool = True          # correlation Gram + greedy pruning
    prune_top_x: object = "top_x"   # None: prune the whole ordered zoo
    # [(op, window)] vs returns: ("corr", 60), ("std", 60) into scratch; ("corr_vol", 60): the
    # feature panel sign(ts_corr(x, R, w)) * x / ts_std(x, w) that the IC, the selection and
    # the composite then run on (C5: ts_corr / ts_std feeding the IC-weighted composite)
    ret_ops: list = field(default_factory=list)
    factor_chunk: int = 0      # ret_ops run over chunks of this many factors (memory)
    composite: object = None   # "zscore" | "rank": weighted composite of the day's selection
    names: object = None       # factor names (composite suffix / prefix rules)
    rank_pass: bool = False    # no op stage ranks X: rank it once (cs_rank2) for the daily IC
    # independent chains on their own HIP streams (engine backend).  Off by default: at C2
    # the overlap gains 2.5 % (87.5 vs 89.7 ms/step) while every stage runs 1.4-3x longer
    # under contention (profiles/r02/streams_ab.log)
    streams: bool = False
    # overlap (round 6, FMX_STEP_OVERLAP=1 for A/B): the rolling set on a side stream for
    # the whole step, next to the one-pass cross-sectional operators -> Gram -> IC chain on
    # the current stream (every operator output in its own buffer).  One shard only.
    overlap: bool = False

    @property
    def lookback(self):
        w = [o[2] for o in self.ops if o[2]] + [w for _, w in self.ret_ops]
        return max(w) if w else 1

    @property
    def halo(self):
        return self.lookback - 1 + max(self.ic_lags)


def factor_names(F):
    """SURVEY 8(d) generator names: g{f//4:03d}_{f:04d}_{suffix}, suffixes cycling."""
    suf = ["eq", "flx", "long", "short", "raw"]
    return [f"g{f // 4:03d}_{f:04d}_{suf[f % 5]}" for f in range(F)]


def workload_config(name):
    if name == "c2":
        return StepConfig()
    if name == "c4":
        # the daily IC from one ranks-only pass (cs_rank2 + the wave IC): 15.1 vs 23.7 ms per
        # 252 dates for the IC kernel that ranks each row itself (profiles/r05)
        return StepConfig(ops=[], ic_lags=(1,), select=False, gram=True, prune_top_x=None, rank_pass=True)
    if name == "c5":
        return StepConfig(ops=[], ic_lags=(1, 2), select=True, gram=False, ret_ops=[("corr_vol", 60)],
                          factor_chunk=100, composite="zscore", rank_pass=True)
    raise ValueError(f"unknown workload {name!r}")


def _op_key(kind, op, w):
    return f"{kind}:{op or ''}:{w or ''}"


def plan_ops(ops, be, fuse=True, zn=True):
    """Group the operator list into launches.  With ``fuse`` and a backend that has the
    multi-output kernels: the rolling set {mean, std, zscore, decay at W; rank at WR}
    becomes one ts_set pass, cs_zscore + market_neutralize one moment pass, cs_rank +
    cs_winsor one histogram pass -- and with ``zn`` all four cross-sectional operators one
    pass over the rows (cs_rank_winsor_zn: the row is read once).  Returns
    [(stage_name, [(kind, op, w), ...])]."""
    left = list(ops)
    stages = []
    quad = [("cs_rank", None, None), ("winsor", None, None), ("cs", "zscore", None), ("cs", "market_neutralize", None)]
    fuse_zn = (fuse and zn and hasattr(be, "cs_rank_winsor_zn") and not getattr(be, "fused_ic", False)
               and all(p in left for p in quad))
    if fuse and hasattr(be, "ts_set"):
        ts = [o for o in left if o[0] == "ts" and o[1] in ("mean", "std", "zscore", "rank", "decay")]
        W = {o[2] for o in ts if o[1] != "rank"}
        WR = {o[2] for o in ts if o[1] == "rank"}
        names = [o[1] for o in ts]
        if len(ts) >= 2 and len(W) <= 1 and len(WR) <= 1 and len(set(names)) == len(names):
            w = next(iter(W)) if W else next(iter(WR))
            wr = next(iter(WR)) if WR else w
            stages.append((f"ts_set:{w}:{wr}", ts))
            left = [o for o in left if o not in ts]
    if fuse_zn:
        left = [o for o in left if o not in quad]
    if fuse and hasattr(be, "cs_rank_winsor"):
        pair = [("cs_rank", None, None), ("winsor", None, None)]
        if all(p in left for p in pair):
            stages.append(("cs_rank_winsor", pair))
            left = [o for o in left if o not in pair]
    stages += [(_op_key(*o), [o]) for o in left]
    if fuse_zn:
        # last: its cs_zscore output is still in its buffer when the Gram reads it
        return stages + [("cs_rank_winsor_zn", quad)]
    if fuse and hasattr(be, "cs_zscore_neutralize"):
        # last: its cs_zscore output is still in its buffer when the Gram reads it
        pair = [("cs", "zscore", None), ("cs", "market_neutralize", None)]
        if all(p in left for p in pair):
            stages = [st for st in stages if st[1][0] not in pair] + [("cs_zscore_neutralize", pair)]
    return stages


def synthetic_panel(D, A, F, device, seed=0, d_lo=0, d_hi=None, halo=0):
    """SURVEY 8(d) generator on the device: X ~ N(0,1) with 1% NaN and 5% of values
    rounded to 1 decimal; R = 0.01 N(0,1) + 0.002 X[d-1,:,0] with 0.5% NaN.  Returns the
    rows [d_lo - halo, d_hi) of the full panel (identical on every rank: the generator is
    seeded per date)."""
    d_hi = D if d_hi is None else d_hi
    lo = max(0, d_lo - halo)
    n = d_hi - lo
    X = torch.empty((F, n, A), dtype=torch.float64, device=device)
    R = torch.empty((n, A), dtype=torch.float64, device=device)
    g = torch.Generator(device=device)
    prev0 = None
    for k, d in enumerate(range(lo, d_hi)):
        g.manual_seed(seed * 1_000_003 + d)
        x = torch.randn((F, A), generator=g, dtype=torch.float64, device=device)
        u = torch.rand((F, A), generator=g, dtype=torch.float64, device=device)
        x = torch.where(u < 0.05, torch.round(x * 10) / 10, x)
        x = torch.where(u > 0.99, torch.full_like(x, float("nan")), x)
        X[:, k] = x
        r = 0.01 * torch.randn((A,), generator=g, dtype=torch.float64, device=device)
        ur = torch.rand((A,), generator=g, dtype=torch.float64, device=device)
        if d > 0:
            if prev0 is None:   # first generated row: regenerate date d-1's factor 0
                g2 = torch.Generator(device=device)
                g2.manual_seed(seed * 1_000_003 + d - 1)
                xp = torch.randn((F, A), generator=g2, dtype=torch.float64, device=device)
                up = torch.rand((F, A), generator=g2, dtype=torch.float64, device=device)
                xp = torch.where(up < 0.05, torch.round(xp * 10) / 10, xp)
                xp = torch.where(up > 0.99, torch.full_like(xp, float("nan")), xp)
                prev0 = xp[0]
            r = r + 0.002 * torch.nan_to_num(prev0)
        r = torch.where(ur < 0.005, torch.full_like(r, float("nan")), r)
        R[k] = r
        prev0 = x[0]
    return X, R, lo


def shard_bounds(D, world, rank, align=1):
    """Owned dates [d_lo, d_hi) of ``rank``: the ceil(D / align) blocks of ``align`` dates
    (the wide Gram's absolute date blocks, E.GRAM_DATE_BLOCK: every block then lies on one
    rank, so its exact partial is the same at any GPU count) split as evenly as whole blocks
    allow -- every rank owns nb // world blocks and the first nb % world ranks one more -- so
    no rank is left without dates while there are at least ``world`` blocks, and
    the larger shares go to the lower ranks, the ones that send a halo (D = 121
    over 2 ranks with a 61-date halo gives rank 0 the 61 dates it must send)."""
    nb = (D + align - 1) // align
    q, rem = divmod(nb, world)
    b0 = rank * q + min(rank, rem)
    b1 = b0 + q + (1 if rank < rem else 0)
    return min(D, b0 * align), min(D, b1 * align)


def shard_align(F):
    """Date alignment of the shards: the wide (F > 256) Gram sums absolute date blocks."""
    return E.GRAM_DATE_BLOCK if F > E.FUSED_GRAM_MAX_F else 1


def check_sharding(D, world, halo, align=1):
    """Every rank must own at least one date, and every rank that sends a halo (all but the
    last) at least ``halo`` dates: its last ``halo`` rows are the next rank's warm-up, and
    with fewer they would include its own not-yet-received halo rows."""
    for r in range(world):
        lo, hi = shard_bounds(D, world, r, align)
        if hi - lo < 1 or (r + 1 < world and hi - lo < halo):
            raise ValueError(f"date sharding of D={D} over {world} ranks: rank {r} owns {hi - lo} dates, "
                             f"needs >= {max(1, halo) if r + 1 < world else 1} (halo {halo})")


class ShardedPanel:
    """A rank's slice of the date axis: owned dates [d_lo, d_hi) plus ``halo`` preceding
    dates, stored contiguously as X[F][halo + own][A].  ``comm`` carries the exchanges
    (factormodeling_amd.comm: TorchComm over RCCL / gloo, or LocalComm for in-process
    shards); by default torch.distributed's process group when one is initialised."""

    def __init__(self, D, A, F, rank=None, world=None, device=None, seed=0, halo=HALO, comm=None, align=None):
        # halo: rolling warm-up + IC lag of the step's longest window (StepConfig.halo)
        if comm is None and world is not None and world > 1:
            from .comm import TorchComm
            comm = TorchComm()
        if comm is not None:
            rank = comm.rank if rank is None else rank
            world = comm.world if world is None else world
            if (rank, world) != (comm.rank, comm.world):
                raise ValueError("rank / world disagree with the comm")
        rank = 0 if rank is None else rank
        world = 1 if world is None else world
        self.comm = comm
        self.D, self.A, self.F = D, A, F
        self.rank, self.world = rank, world
        self.align = shard_align(F) if align is None else align
        check_sharding(D, world, halo, self.align)
        self.d_lo, self.d_hi = shard_bounds(D, world, rank, self.align)
        self.halo = halo if rank > 0 else 0
        self.halo_len = halo
        self.device = device
        Xo, Ro, lo = synthetic_panel(D, A, F, device, seed, self.d_lo, self.d_hi, 0)
        assert lo == self.d_lo
        if self.halo:
            # halo rows start as NaN: only exchange_halo() fills them (a skipped exchange
            # shows up as NaN rolling outputs on the first owned dates)
            self.X = torch.full((F, self.halo + Xo.shape[1], A), float("nan"), dtype=Xo.dtype, device=device)
            self.R = torch.full((self.halo + Ro.shape[0], A), float("nan"), dtype=Ro.dtype, device=device)
            self.X[:, self.halo:] = Xo
            self.R[self.halo:] = Ro
            del Xo, Ro
        else:
            self.X, self.R = Xo, Ro
        self.own = self.d_hi - self.d_lo

    def exchange_halo_start(self):
        """Post the halo exchange: send my last ``halo`` owned dates to rank+1, receive
        rank-1's (RCCL point-to-point over xGMI; gloo on CPU; device copies in-process).
        Asynchronous: work that needs no halo row runs while the transfer is in flight;
        exchange_halo_finish() waits and writes the received rows into the halo."""
        if self.world == 1:
            return None
        H = self.halo_len
        # one slab per direction: the last H owned dates of every factor with the returns
        # as factor F ([F + 1][H][A]); the rank's send and receive are one p2p group
        sends, recvs, bufs = [], [], []
        if self.rank + 1 < self.world:
            slab = torch.cat([self.X[:, -H:], self.R[-H:].unsqueeze(0)], dim=0)
            bufs.append(slab)
            sends.append((slab, self.rank + 1))
        recv = None
        if self.rank > 0:
            recv = torch.empty((self.F + 1, self.halo, self.A), dtype=self.X.dtype, device=self.X.device)
            recvs.append((recv, self.rank - 1))
        if hasattr(self.comm, "exchange"):
            reqs = self.comm.exchange(sends, recvs)
        else:
            reqs = [self.comm.isend(t, d) for t, d in sends] + [self.comm.irecv(t, s) for t, s in recvs]
        return reqs, recv, bufs

    def exchange_halo_finish(self, handle):
        if handle is None:
            return
        reqs, recv, _ = handle
        for r in reqs:
            r.wait()
        if recv is not None:
            self.X[:, :self.halo] = recv[:self.F]
            self.R[:self.halo] = recv[self.F]

    def exchange_halo(self):
        self.exchange_halo_finish(self.exchange_halo_start())


class EngineBackend:
    """The product compute backend: libfmx kernels on the local GPU."""

    @staticmethod
    def ts_set(X, ops, outs):
        """ops: [(kind, op, w)] of the rolling set; outs: one buffer per op."""
        W = {w for _, op, w in ops if op != "rank"}
        WR = {w for _, op, w in ops if op == "rank"}
        w = next(iter(W)) if W else next(iter(WR))
        wr = next(iter(WR)) if WR else w
        E.ts_set(X, {op: y for (_, op, _), y in zip(ops, outs)}, w, wr)

    @staticmethod
    def cs_zscore_neutralize(X, outs):
        """Returns cs_zscore's row stats (mean, std) for the Gram."""
        _, _, stats = E.cs_zscore_neutralize(X, outs[0], outs[1], with_stats=True)
        return stats

    @staticmethod
    def cs_rank_winsor(X, outs, rank2=None):
        """``rank2``: also the doubled ranks the daily IC starts from."""
        E.cs_rank_winsor(X, 0.01, 0.99, outs[0], outs[1], rank2=rank2)

    @staticmethod
    def cs_rank_winsor_zn(X, outs, rank2=None, dates=None):
        """cs_rank, cs_winsor, cs_zscore and market_neutralize of the rows in one pass
        (``dates`` = (d0, d1): only those dates' rows)."""
        E.cs_rank_winsor_zn(X, 0.01, 0.99, *outs, rank2=rank2, dates=dates)

    # the fused pass and the ranks-only pass take date sub-ranges (the sharded step's plan)
    zn_dates = True

    ranked_ic_max_a = E.RANKED_IC_MAX_A

    # ranks-only pass + wave IC vs the standalone IC kernel at C5's 10,000 assets:
    # 142 + 43 ms vs 226 ms (profiles/r02/c5_h6.log; was 420 + 76 ms before the rank
    # kernel's LDS-aware launch bounds and 1024-thread rows, c5_h1.log)
    rank_pass_max_a = int(os.environ.get("FMX_RANK_PASS_MAX_A", "16384"))

    @staticmethod
    def cs_rank2(X, rank2, dates=None):
        """The doubled ranks alone (no operator output): the IC's rank pass."""
        E.cs_rank2(X, rank2, dates=dates)

    # the daily IC fused into the rank pass (fmx_cs_rank_winsor_ic: the ranks never leave
    # the CU).  Off by default: at C2 it measured 37.4 ms against 21.1 + 8.8 ms for the rank
    # pass + k_ic_wave pair (the IC tail lengthens every row's barrier chain at the 3 rows
    # per CU the LDS admits).  FMX_FUSED_IC=1 selects it (A/B)
    fused_ic = os.environ.get("FMX_FUSED_IC", "0") == "1"

    @staticmethod
    def cs_rank_winsor_ic(X, R, lags, outs, rank2):
        """cs_rank + cs_winsor into ``outs`` (None: ranks only) and the daily IC records."""
        if outs is None:
            return E.cs_rank_winsor_ic(X, R, lags, ranks_only=True, rank2=rank2)[2]
        return E.cs_rank_winsor_ic(X, R, lags, 0.01, 0.99, outs[0], outs[1], rank2=rank2)[2]

    def op(self, kind, op, w, X, out):
        if kind == "ts":
            return E.ts(op, X, w, None, out=out)
        if kind == "cs_rank":
            return E.cs_rank(X, out=out)
        if kind == "cs":
            return E.cs_moment(op, X, out=out)
        if kind == "winsor":
            return E.cs_quantile_op("winsor", X, 0.01, 0.99, out=out)
        raise ValueError(kind)

    @staticmethod
    def cs_zscore_stats(X, out):
        """cs_zscore that also returns the per-row (mean, std) the Gram reuses."""
        return E.cs_moment_stats("zscore", X, out=out)

    @staticmethod
    def corr_gram_exact(X, d0, d1, stats=None, z=None):
        """Exact fixed-point Gram partials over dates [d0, d1) (F <= 256): from ``z``, the
        step's cs_zscore output, when given, else from X with the row stats."""
        if z is not None:
            return E.gram_exact(z, None, d0, d1)
        if stats is None:
            _, stats = E.cs_moment_stats("stats", X)
        return E.gram_exact(X, stats, d0, d1)

    gram_exact_finalize = staticmethod(E.gram_exact_finalize)

    @staticmethod
    def corr_gram_wide_exact(X, d0, d1, d_origin, stats=None):
        """Exact fixed-point partials of the wide Gram (any F) over local dates [d0, d1);
        local row 0 is absolute date ``d_origin`` (slices are absolute date blocks)."""
        return E.gram_direct_exact(X, d0, d1, d_origin, stats)

    @staticmethod
    def corr_gram(X, d0, d1, stats=None, z=None):
        """G, N over dates [d0, d1): fused single pass for F <= 256 (from ``z``, the
        step's cs_zscore output, when given), else the wide tiles straight from X."""
        if X.shape[0] <= E.FUSED_GRAM_MAX_F:
            # the z input needs the default kernel; the A/B switches take the stats path
            ab = os.environ.get("FMX_GRAM_SINGLE_BUFFER") or os.environ.get("FMX_GRAM_MASK_MFMA")
            if z is not None and not ab:
                return E.gram_fused(z, None, d0, d1)
            if stats is None:
                _, stats = E.cs_moment_stats("stats", X)
            return E.gram_fused(X, stats, d0, d1)
        return E.gram_wide(X, d0, d1)

    @staticmethod
    def ts_corr_into(X, R, w, out):
        E.ts_corr(X, R, w, out=out)

    @staticmethod
    def corr_vol_feature(X, C, w, out):
        E.corr_vol_feature(X, C, w, out=out)

    @staticmethod
    def corr_feature_into(X, R, w, out, corr_out=None):
        E.corr_feature(X, R, w, out=out, corr_out=corr_out)

    wcomp = staticmethod(E.wcomp)
    ic_daily = staticmethod(E.ic_daily)
    ic_window = staticmethod(E.ic_window)
    select_icir_top = staticmethod(E.select_icir_top)
    zscore_exposures = staticmethod(E.zscore_exposures)
    gram = staticmethod(E.gram)
    greedy_prune = staticmethod(E.greedy_prune)


ENGINE = EngineBackend()


# the per-date stages a step runs while the halo exchange is in flight (their owned-date
# results read no halo row); the Gram follows them on its z-score
EARLY_STAGES = ("cs_zscore_neutralize", "cs_rank_winsor_zn")


def _stage_stream(name, streams):
    """The stream a planned stage runs on (None: the current stream).  Three independent
    chains of the step: the rolling set (streams[0]); cs_zscore + market_neutralize, whose
    row stats feed the Gram (streams[1]); the rank pass, whose ranks feed the daily IC
    (current stream)."""
    if not streams:
        return None
    if name.startswith("ts_set:"):
        return streams[0]
    if name == "cs_zscore_neutralize":
        return streams[1]
    return None


def run_ops(X, cfg: StepConfig, bufs=None, timers=None, be=ENGINE, collect=None, own=slice(None), side=None,
            streams=None, only=None, zn=True):
    """Operator set over the local panel (halo rows included as warm-up), as planned by
    ``plan_ops``; every operator writes its own output buffer (``bufs``: a list of tensors
    shaped like X, reused across steps).  Sequentially, stages share the buffers (as many
    as the widest fused launch); with ``streams`` (stages running concurrently) every
    stage gets its own.  ``collect`` (a dict) receives a copy of every operator's
    owned-date output (tests only); ``side`` (a dict) receives by-products later stages
    reuse (cs_zscore's row stats; "rank2", the doubled ranks of X, written into
    side["rank2_buf"] when it fits).  ``only``: run just the stages it accepts (by name)."""
    stages = plan_ops(cfg.ops, be, cfg.fuse, zn=zn and not cfg.streams)
    offs, need = [], 0
    for _, ops in stages:
        offs.append(need if streams else 0)
        need = need + len(ops) if streams else max(need, len(ops))
    bufs = list(bufs or [])
    while len(bufs) < need:
        bufs.append(torch.empty_like(X))
    for (name, ops), off in zip(stages, offs):
        if only is not None and not only(name):
            continue
        outs = bufs[off:off + len(ops)]
        st = _stage_stream(name, streams)
        ctx = torch.cuda.stream(st) if st is not None else contextlib.nullcontext()
        with ctx:
            if side is not None and any(o is side.get("zscore") for o in outs):
                side.pop("zscore")                   # about to be overwritten
            _run_stage(name, ops, outs, X, be, side, timers, collect, own)
    return bufs


def _run_stage(name, ops, outs, X, be, side, timers, collect, own):
    """One planned stage (fused or single operator) on the current stream."""
    t0 = _ev(timers)
    if name.startswith("ts_set:"):
        be.ts_set(X, ops, outs)
    elif name == "cs_zscore_neutralize":
        st = be.cs_zscore_neutralize(X, outs)
        if side is not None:
            side["stats"] = st
            side["zscore"] = outs[0]                # the Gram's z (valid until the buffer is reused)
    elif name == "cs_rank_winsor_zn":
        rk = None
        if side is not None and X.shape[2] <= getattr(be, "ranked_ic_max_a", 0):
            rk = side.get("rank2_buf")
            if rk is None or tuple(rk.shape) != tuple(X.shape):
                rk = torch.empty(X.shape, dtype=E.RANK2_DTYPE, device=X.device)
            side["rank2"] = rk
        zd = side.get("zn_dates") if side is not None else None
        if zd is not None:
            # sharded: the owned dates now (the halo exchange is in flight); the doubled
            # ranks of the halo rows follow once it lands (run_step)
            be.cs_rank_winsor_zn(X, outs, rank2=rk, dates=zd)
            if rk is not None:
                side["rank2_halo"] = (0, zd[0])
        else:
            be.cs_rank_winsor_zn(X, outs, rank2=rk)
        if side is not None:
            side["stats"] = None
            side["zscore"] = outs[2]                # the Gram's z (valid until the buffer is reused)
    elif name == "cs_rank_winsor":
        if side is not None and X.shape[2] <= getattr(be, "ranked_ic_max_a", 0):
            # the ranks of X also feed the daily IC (no second ranking of the panel)
            rk = side.get("rank2_buf")
            if rk is None or tuple(rk.shape) != tuple(X.shape):
                rk = torch.empty(X.shape, dtype=E.RANK2_DTYPE, device=X.device)
            side["rank2"] = rk
            if _fused_ic(be, side):
                # ... inside the same pass: the daily IC records of every row
                side["daily"] = be.cs_rank_winsor_ic(X, side["R"], side["lags"], outs, rk)
                name = "cs_rank_winsor_ic"
            else:
                be.cs_rank_winsor(X, outs, rank2=rk)
        else:
            be.cs_rank_winsor(X, outs)
    else:
        kind, op, w = ops[0]
        if side is not None and (kind, op) == ("cs", "zscore") and hasattr(be, "cs_zscore_stats"):
            _, side["stats"] = be.cs_zscore_stats(X, outs[0])
        else:
            be.op(kind, op, w, X, outs[0])
    _rec(timers, name, t0)
    if collect is not None:
        fs = collect.get("_factors")             # full-size tests: only a sample of factors
        for o, y in zip(ops, outs):
            collect[_op_key(*o)] = (y if fs is None else y[fs])[:, own].clone()


def _fused_ic(be, side):
    """The backend fuses the daily IC into the rank pass for this step's lags."""
    return (getattr(be, "fused_ic", False) and hasattr(be, "cs_rank_winsor_ic") and side.get("R") is not None
            and 1 <= len(side.get("lags") or ()) <= 2)


def _ev(timers):
    if timers is None or not torch.cuda.is_available():
        return None
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return e


def _rec(timers, name, t0):
    if timers is None or t0 is None:
        return
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    timers.append((name, t0, e))


def run_ret_ops(sp, cfg, timers=None, be=ENGINE, collect=None):
    """Operators against the returns over factor chunks of ``cfg.factor_chunk`` (a
    full-size output per operator would not fit next to a 100 GB panel): ("corr", w) /
    ("std", w) write reused chunk buffers; ("corr_vol", w) -- C5 -- writes the chunk of the
    feature panel sp.feature = sign(ts_corr(x, R, w)) * x / ts_std(x, w) in one pass
    (fmx_ts_corr_feature; a backend without it: ts_corr into a chunk buffer, then
    fmx_ts_corr_vol_feature), which the rest of the step runs on."""
    F = sp.X.shape[0]
    fused = lambda op, w: op == "corr_vol" and hasattr(be, "corr_feature_into") and w <= getattr(  # noqa: E731
        be, "corr_feature_max_w", E.CORR_FEATURE_MAX_W)
    want_corr = collect is not None and collect.get("_factors") is None
    if all(fused(op, w) for op, w in cfg.ret_ops) and not want_corr:
        # every op is the one-pass corr -> feature writing straight into sp.feature: no
        # scratch, so no chunks -- one launch over all factors (five 100-factor launches
        # each ended on a part-filled round of workgroups)
        fc, bufs = F, [None] * len(cfg.ret_ops)
    else:
        fc = cfg.factor_chunk or F
        n = min(fc, F)
        bufs = getattr(sp, "ret_bufs", None)
        if bufs is None or bufs[0].shape[0] != n or len(bufs) != len(cfg.ret_ops):
            bufs = [torch.empty((n,) + tuple(sp.X.shape[1:]), dtype=sp.X.dtype, device=sp.X.device)
                    for _ in cfg.ret_ops]
            sp.ret_bufs = bufs
    if any(op == "corr_vol" for op, _ in cfg.ret_ops) and getattr(sp, "feature", None) is None:
        sp.feature = torch.empty_like(sp.X)
    for f0 in range(0, F, fc):
        f1 = min(F, f0 + fc)
        Xc = sp.X[f0:f1]
        for (op, w), buf in zip(cfg.ret_ops, bufs):
            out = buf[: f1 - f0] if buf is not None else None
            t0 = _ev(timers)
            if fused(op, w):
                # one pass: the corr stays in registers (written only when collected)
                want = want_corr
                be.corr_feature_into(Xc, sp.R, w, sp.feature[f0:f1], out if want else None)
                _rec(timers, f"ret:corr_vol:{w}", t0)
                if want:
                    collect.setdefault(f"ret:corr:{w}", []).append(out[:, sp.halo:].clone())
                continue
            if op in ("corr", "corr_vol"):
                be.ts_corr_into(Xc, sp.R, w, out)
            else:
                be.op("ts", op, w, Xc, out)
            _rec(timers, f"ret:{'corr' if op == 'corr_vol' else op}:{w}", t0)
            if collect is not None and collect.get("_factors") is None:
                collect.setdefault(f"ret:{'corr' if op == 'corr_vol' else op}:{w}", []).append(out[:, sp.halo:].clone())
            if op == "corr_vol":
                t0 = _ev(timers)
                be.corr_vol_feature(Xc, out, w, sp.feature[f0:f1])
                _rec(timers, f"ret:cvf:{w}", t0)
    if collect is not None and getattr(sp, "feature", None) is not None:
        fs = collect.get("_factors")
        collect["feature"] = (sp.feature if fs is None else sp.feature[fs])[:, sp.halo:].clone()


def _step_panel(sp, cfg):
    """The panel the IC, the selection and the composite run on: the C5 feature panel
    when the step builds one, else the factor panel itself."""
    if any(op == "corr_vol" for op, _ in cfg.ret_ops):
        return sp.feature
    return sp.X


def run_step(sp: ShardedPanel, cfg: StepConfig, timers=None, be=ENGINE, collect=None):
    """One pass of the hot path.  Returns (selected weights [J][F] (every rank holds the
    full result; None without selection), kept factor list (None without the Gram)).
    ``collect`` (tests) receives intermediate results."""
    # "rank2" is filled when this step ranks X; "daily" when the IC ran inside the rank pass
    side = {"rank2_buf": getattr(sp, "rank2", None), "R": sp.R, "lags": tuple(cfg.ic_lags)}
    streams = None
    early = not cfg.streams
    # the four cross-sectional operators in one pass.  Sharded, the pass runs on the owned
    # dates while the halo exchange is in flight (every output row is per-date), and the
    # doubled ranks of the halo rows -- the first owned dates' daily IC reads exposures at
    # t - lag -- follow once the exchange lands (fmx_cs_rank2_dates).  A backend without
    # date ranges takes the two-pass form sharded (cs_zscore + neutralize in front of the
    # exchange, rank + winsor after it)
    zn = sp.halo == 0 or (getattr(be, "zn_dates", False) and sp.X.shape[2] <= getattr(be, "ranked_ic_max_a", 0))
    if zn and sp.halo > 0:
        side["zn_dates"] = (sp.halo, sp.X.shape[1])
    early_names = EARLY_STAGES
    overlap = (cfg.overlap and not cfg.streams and cfg.ops and hasattr(be, "ts_set") and sp.X.is_cuda
               and sp.world == 1)
    side_st = None
    if overlap:
        # the rolling set first, on its own stream (it reads only X); its outputs get their
        # own buffers (run_ops with streams: one buffer range per stage).  (Enqueued behind
        # the cross-sectional pass instead, it overlapped the Gram: 69.7 / 71.0 vs 67.8 / 67.6 ms)
        side_st = getattr(sp, "side_stream", None)
        if side_st is None:
            side_st = sp.side_stream = torch.cuda.Stream(sp.X.device)
        side_st.wait_stream(torch.cuda.current_stream(sp.X.device))
        sp.bufs = run_ops(sp.X, cfg, getattr(sp, "bufs", None), timers=timers, be=be, collect=collect,
                          side=side, streams=[side_st], only=lambda n: n.startswith("ts_set:"), zn=zn)
    t0 = _ev(timers)
    halo = sp.exchange_halo_start()
    _rec(timers, "halo", t0)
    GN = None
    if early:
        # while the halo is in flight: the stages whose owned-date results read no halo
        # row -- cs_zscore + market_neutralize (per-date rows) and the Gram over the owned
        # dates (from that z-score).  They also process the halo rows, whose outputs are
        # not owned (stale until the exchange lands: the same data every step).
        if cfg.ops:
            # (overlap: the stream-aware buffer ranges, so no stage shares the rolling set's)
            sp.bufs = run_ops(sp.X, cfg, getattr(sp, "bufs", None), timers=timers, be=be, collect=collect,
                              own=slice(sp.halo, None), side=side, streams=[side_st] if overlap else None,
                              only=lambda n: n in early_names, zn=zn)
        if cfg.gram and hasattr(be, "corr_gram"):
            t0 = _ev(timers)
            GN = gram_partials(sp, be, side)
            _rec(timers, "gram", t0)
    t0 = _ev(timers)
    sp.exchange_halo_finish(halo)
    _rec(timers, "halo_wait", t0)
    if side.get("rank2_halo") is not None:
        t0 = _ev(timers)
        be.cs_rank2(sp.X, side["rank2"], dates=side.pop("rank2_halo"))
        _rec(timers, "rank2_halo", t0)
    if cfg.streams and cfg.ops and hasattr(be, "ts_set") and sp.X.is_cuda:
        # fork: the rolling set and the cs_zscore -> Gram chain on side streams, the rank
        # pass -> IC -> selection chain on the current one; joined before the Gram sum
        streams = getattr(sp, "streams", None)
        if streams is None:
            streams = sp.streams = [torch.cuda.Stream(sp.X.device) for _ in range(2)]
        main = torch.cuda.current_stream(sp.X.device)
        for st in streams:
            st.wait_stream(main)
    if cfg.ops:
        if overlap:                               # the rolling set is already on its stream
            rest = lambda n: n not in early_names and not n.startswith("ts_set:")  # noqa: E731
            sp.bufs = run_ops(sp.X, cfg, getattr(sp, "bufs", None), timers=timers, be=be, collect=collect,
                              own=slice(sp.halo, None), side=side, streams=[side_st], only=rest, zn=zn)
        else:
            sp.bufs = run_ops(sp.X, cfg, getattr(sp, "bufs", None), timers=timers, be=be, collect=collect,
                              own=slice(sp.halo, None), side=side, streams=streams,
                              only=(lambda n: n not in early_names) if early else None, zn=zn)
    if streams is not None and cfg.gram and hasattr(be, "corr_gram"):
        with torch.cuda.stream(streams[1]):       # right behind cs_zscore's row stats
            t0 = _ev(timers)
            GN = gram_partials(sp, be, side)
            _rec(timers, "gram", t0)
    if cfg.ret_ops:
        run_ret_ops(sp, cfg, timers, be, collect)
    Xs = _step_panel(sp, cfg)
    if Xs is not sp.X:
        # the ranks / fused IC records of the operator stage are of X, not of the feature
        # panel the IC runs on: rank the feature panel itself below
        side.pop("rank2", None)
        side.pop("daily", None)
    if (cfg.rank_pass and side.get("rank2") is None and hasattr(be, "cs_rank2")
            and sp.A <= getattr(be, "rank_pass_max_a", 0)):
        # no operator ranked X this step: one ranks-only pass feeds the IC (inside the pass
        # when the backend fuses it, else the wave IC from the ranks)
        t0 = _ev(timers)
        rk = getattr(sp, "rank2", None)
        if rk is None:
            rk = torch.empty(Xs.shape, dtype=E.RANK2_DTYPE, device=Xs.device)
        side["rank2"] = rk
        if _fused_ic(be, side):
            side["daily"] = be.cs_rank_winsor_ic(Xs, sp.R, side["lags"], None, rk)
            _rec(timers, "rank_ic", t0)
        else:
            be.cs_rank2(Xs, rk)
            _rec(timers, "rank2", t0)
    # daily IC for owned dates (halo provides the lagged rows)
    t0 = _ev(timers)
    lags = tuple(cfg.ic_lags)
    if side.get("daily") is not None:
        sp.rank2 = side["rank2"]
        daily = side["daily"][:, :, :, sp.halo:]                        # made by the rank pass
        t0 = None
    elif side.get("rank2") is not None:
        sp.rank2 = side["rank2"]                                        # buffer reused next step
        daily = be.ic_daily(Xs, sp.R, lags, rank2=sp.rank2)[:, :, :, sp.halo:]
    else:
        daily = be.ic_daily(Xs, sp.R, lags)[:, :, :, sp.halo:]        # [L][4][F][own]
    _rec(timers, "ic_daily", t0)
    t0 = _ev(timers)
    L = len(lags)
    if sp.world > 1:
        # every rank pads its owned dates to the longest shard; each slice is placed by
        # its owner's bounds
        spans = [shard_bounds(sp.D, sp.world, r, getattr(sp, "align", 1)) for r in range(sp.world)]
        per = max(hi - lo for lo, hi in spans)
        pad = torch.zeros((L, 4, sp.F, per), dtype=daily.dtype, device=daily.device)
        pad[..., :daily.shape[3]] = daily
        parts = sp.comm.all_gather(pad)
        full = torch.cat([p[..., :hi - lo] for p, (lo, hi) in zip(parts, spans)], dim=3).contiguous()
    else:
        full = daily.contiguous()
    _rec(timers, "allgather_ic", t0)
    t0 = _ev(timers)
    D = full.shape[3]
    summ = be.ic_window(full[0].contiguous(), [0], [D])                # full-sample metrics
    w = win = None
    if cfg.select:
        W = cfg.sel_window
        proc = list(range(W, D - 1))
        win = be.ic_window(full[L - 1].contiguous(), [i - W + 1 for i in proc], proc)
        order, w = be.select_icir_top(win, True, cfg.icir_threshold, cfg.top_x)
    _rec(timers, "select", t0)
    comp = None
    if cfg.composite and w is not None:
        t0 = _ev(timers)
        comp = weighted_composite_step(sp, cfg, w, be, Xs)
        _rec(timers, "composite", t0)
    if streams is not None:                       # join
        main = torch.cuda.current_stream(sp.X.device)
        for st in streams:
            main.wait_stream(st)
    kept = C = None
    if cfg.gram:
        # correlation Gram over owned dates, summed over ranks in rank order
        t0 = _ev(timers)
        made = GN is not None
        if made:
            for T in GN[1]:                       # made on streams[1]: now used on this one
                if T.is_cuda:
                    T.record_stream(torch.cuda.current_stream(T.device))
        else:
            GN = gram_partials(sp, be, side)
        G, N = gram_total(sp, be, GN)
        C = torch.where(N > 0, G / N.clamp_min(1.0), torch.zeros_like(G))
        _rec(timers, "gram_sum" if made else "gram", t0)
        t0 = _ev(timers)
        rir = summ[0, :, 3]
        full_order = torch.argsort(torch.nan_to_num(rir, nan=-np.inf), descending=True, stable=True)
        top = cfg.top_x if cfg.prune_top_x == "top_x" else cfg.prune_top_x
        kept = be.greedy_prune(C, full_order.cpu().numpy(), cfg.prune_rho, top)
        _rec(timers, "prune", t0)
    if side_st is not None:                       # join the rolling set
        torch.cuda.current_stream(sp.X.device).wait_stream(side_st)
    if collect is not None:
        collect.update(daily=full, summ=summ, win=win, C=C, comp=comp)
    return w, kept


def gram_partials(sp, be, side):
    """This rank's share of the factor Gram over its owned dates: ("exact", (limbs, counts))
    -- integer fixed-point partials whose sum over ranks is independent of the GPU count
    (F <= 256: gram_exact's per-date units; wider: gram_direct_exact's absolute date blocks,
    the shards aligned to them) -- or ("float", (G, N)) for backends without either."""
    d0, d1 = sp.halo, sp.X.shape[1]
    if hasattr(be, "corr_gram_exact") and sp.F <= E.FUSED_GRAM_MAX_F:
        return "exact", be.corr_gram_exact(sp.X, d0, d1, side.get("stats"), side.get("zscore"))
    if hasattr(be, "corr_gram_wide_exact") and sp.d_lo % getattr(sp, "align", 1) == 0 \
            and getattr(sp, "align", 1) % E.GRAM_DATE_BLOCK == 0:
        return "exact", be.corr_gram_wide_exact(sp.X, d0, d1, sp.d_lo - sp.halo, side.get("stats"))
    if hasattr(be, "corr_gram"):
        return "float", be.corr_gram(sp.X, d0, d1, side.get("stats"), side.get("zscore"))
    Z, M = be.zscore_exposures(sp.X[:, d0:].contiguous())
    return "float", be.gram(Z, M)


def gram_total(sp, be, part):
    """G, N over all ranks' dates.  Exact partials: int64 all-reduce (RCCL over xGMI; the
    integer sum is the same in any order) then finalize -- the same bits at 1, 2, 4 or 8
    GPUs, so the kept set never depends on the GPU count.  Float partials: rank-ordered sum
    (identical on every rank of one run)."""
    kind, (a, b) = part
    if kind == "exact":
        if sp.world > 1:
            sp.comm.all_reduce_sum(a)
            sp.comm.all_reduce_sum(b)
        return be.gram_exact_finalize(a, b)
    if sp.world > 1:
        a, b = ordered_sum(a, sp.comm), ordered_sum(b, sp.comm)
    return a, b


def weighted_composite_step(sp, cfg, w, be=ENGINE, X=None):
    """weighted_composite_factor (composite_factor.py:220-342) of each processed day's
    selection over this rank's owned dates of ``X`` (default the factor panel; C5: its
    feature panel): the day's selected columns, pooled suffix percentiles, prefix proxies,
    group weights, z-score / rank, demeaning."""
    from .composite_factor import weighted_plan
    X = sp.X if X is None else X
    W = cfg.sel_window
    D = w.shape[0] + W + 1
    proc = np.arange(W, D - 1)
    local = proc - sp.d_lo + sp.halo                    # rows of the local panel
    own = (proc >= sp.d_lo) & (proc < sp.d_hi)
    pdate = np.where(own, local, -1)
    names = cfg.names or factor_names(sp.F)
    if hasattr(be, "weighted_composite"):               # the oracle (tests)
        return be.weighted_composite(X, names, pdate, w, cfg.composite)
    plan = weighted_plan(pdate, w.cpu().numpy(), names)
    return be.wcomp(X, plan, cfg.composite)


def ordered_sum(T, comm):
    """Sum of every rank's ``T`` in rank order (all-gather + sequential adds): identical on
    every rank, but a different rounding of the sum at each GPU count.  Only backends
    without the exact Gram partials use it (the CPU oracle backend in the gloo tests)."""
    parts = comm.all_gather(T.contiguous())
    acc = parts[0].clone()
    for p in parts[1:]:
        acc += p
    return acc


def _ev_ok():
    return torch.cuda.is_available()


def stage_times(timers):
    torch.cuda.synchronize()
    out = {}
    for name, a, b in timers:
        out[name] = out.get(name, 0.0) + a.elapsed_time(b)
    return out
