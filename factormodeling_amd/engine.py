"""Device-tensor API over libfmx: every function takes/returns torch CUDA (HIP) tensors
laid out ``[F][D][A]`` float64 (asset fastest) and launches the gfx950 kernels on the
current torch stream.  Shapes are validated on the host before any launch.

This is the layer the drop-in pandas modules, the benchmark and the date-sharded
multi-GPU driver are built on.
"""
from __future__ import annotations

import os
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import CS, CSREG, EW, GROUP, RANK, TS, call, ptr, stream_ptr

F64 = torch.float64


def _check_panel(X, name="X"):
    if not isinstance(X, torch.Tensor) or X.device.type != "cuda":
        raise _lib.FmxError(f"{name} must be a HIP device tensor")
    if X.dtype != F64:
        raise _lib.FmxError(f"{name} must be float64")
    if X.dim() != 3:
        raise _lib.FmxError(f"{name} must be [F][D][A]")
    if not X.is_contiguous():
        raise _lib.FmxError(f"{name} must be contiguous")


def _check_present(present, D, A):
    if present is None:
        return None
    if present.dtype != torch.uint8 or tuple(present.shape) != (D, A) or not present.is_contiguous():
        raise _lib.FmxError("present must be a contiguous uint8 [D][A] device tensor")
    return present


def as3(X):
    return X if X.dim() == 3 else X.unsqueeze(0)


def empty_like(X):
    return torch.empty_like(X)


# ----------------------------------------------------------------------------- time series
def ts(op: str, X, window: int, present=None, out=None):
    X = as3(X)
    _check_panel(X)
    F, D, A = X.shape
    _check_present(present, D, A)
    Y = _out(X, out)
    call("fmx_ts_op", TS[op], ptr(X), ptr(Y), F, D, A, A, int(window), ptr(present), stream_ptr())
    return Y


TS_SET = ("mean", "std", "zscore", "rank", "decay")


def ts_set(X, outs: dict, window: int, rank_window: int, present=None):
    """Fused rolling set (fmx_ts_set): ``outs`` maps a subset of TS_SET to output
    tensors shaped like X; mean/std/zscore/decay use ``window``, rank ``rank_window``."""
    X = as3(X)
    _check_panel(X)
    F, D, A = X.shape
    _check_present(present, D, A)
    bad = set(outs) - set(TS_SET)
    if bad:
        raise ValueError(f"ts_set: unsupported ops {sorted(bad)}")
    ps = [ptr(_out(X, outs[k])) if k in outs else None for k in TS_SET]
    call("fmx_ts_set", ptr(X), *ps, F, D, A, A, int(window), int(rank_window), ptr(present), stream_ptr())
    return outs


def ts_corr(X, Ycol, window: int, present=None, out=None):
    X = as3(X)
    _check_panel(X)
    F, D, A = X.shape
    _check_present(present, D, A)
    if Ycol.dim() == 2:
        if tuple(Ycol.shape) != (D, A):
            raise _lib.FmxError("Ycol must be [D][A] or [F][D][A]")
        ystride = 0
    else:
        if tuple(Ycol.shape) != (F, D, A):
            raise _lib.FmxError("Ycol must be [D][A] or [F][D][A]")
        ystride = D * A
    Ycol = Ycol.contiguous()
    out = _out(X, out)
    call("fmx_ts_corr", ptr(X), ptr(Ycol), ptr(out), F, D, A, A, ystride, int(window), ptr(present), stream_ptr())
    return out


# fmx_ts_corr_feature keeps the window's reciprocal table in LDS up to this window
# (ts_ops.hip TSC_MAXW); longer windows take ts_corr + corr_vol_feature
CORR_FEATURE_MAX_W = 4096


def corr_feature(X, Ycol, window: int, out=None, corr_out=None):
    """C5's feature sign(ts_corr(X, Ycol, window)) * (X / ts_std(X, window)) in one pass
    (fmx_ts_corr_feature): bit-identical to ts_corr + corr_vol_feature, without the corr
    panel's round trip.  ``corr_out`` (optional) also receives the corr.  Dense panels."""
    X = as3(X)
    _check_panel(X)
    F, D, A = X.shape
    if Ycol.dim() == 2:
        if tuple(Ycol.shape) != (D, A):
            raise _lib.FmxError("Ycol must be [D][A] or [F][D][A]")
        ystride = 0
    else:
        if tuple(Ycol.shape) != (F, D, A):
            raise _lib.FmxError("Ycol must be [D][A] or [F][D][A]")
        ystride = D * A
    Ycol = Ycol.contiguous()
    out = _out(X, out)
    if corr_out is not None:
        corr_out = _out(X, corr_out)
    call("fmx_ts_corr_feature", ptr(X), ptr(Ycol), ptr(corr_out), ptr(out), F, D, A, A, ystride, int(window),
         stream_ptr())
    return out


def corr_vol_feature(X, C, window: int, out=None):
    """C5's feature sign(C) * (X / ts_std(X, window)) (fmx_ts_corr_vol_feature); C is
    ts_corr(X, R, window) of the same rows (same shape as X)."""
    X = as3(X)
    _check_panel(X)
    C = as3(C)
    _check_panel(C, "C")
    if C.shape != X.shape:
        raise _lib.FmxError("C must be shaped like X")
    F, D, A = X.shape
    out = _out(X, out)
    call("fmx_ts_corr_vol_feature", ptr(X), ptr(C), ptr(out), F, D, A, A, int(window), stream_ptr())
    return out


def ts_regression(Yv, Xv, valid, window: int, rettype: int):
    D, A = Yv.shape
    if tuple(Xv.shape) != (D, A) or tuple(valid.shape) != (D, A) or valid.dtype != torch.uint8:
        raise _lib.FmxError("ts_regression: shape mismatch")
    out = torch.empty_like(Yv)
    call("fmx_ts_regression", ptr(Yv), ptr(Xv), ptr(valid), ptr(out), D, A, A, int(window), int(rettype),
         stream_ptr())
    return out


# ----------------------------------------------------------------------------- cross section
def _out(X, out):
    if out is None:
        return torch.empty_like(X)
    if out.shape != X.shape or out.dtype != X.dtype or not out.is_contiguous() or out.data_ptr() == X.data_ptr():
        raise _lib.FmxError("out must be a distinct contiguous tensor shaped like X")
    return out


def cs_moment(op: str, X, present=None, out=None):
    X = as3(X)
    _check_panel(X)
    F, D, A = X.shape
    _check_present(present, D, A)
    Y = _out(X, out)
    call("fmx_cs_moment", CS[op], ptr(X), ptr(Y), F, D, A, A, ptr(present), stream_ptr())
    return Y


def cs_moment_stats(op: str, X, present=None, out=None):
    """fmx_cs_moment plus the per-row (mean, std ddof=0) [F][D][2]; op 'stats' returns
    (None, stats) without writing an output panel."""
    X = as3(X)
    _check_panel(X)
    F, D, A = X.shape
    _check_present(present, D, A)
    Y = None if op == "stats" else _out(X, out)
    stats = torch.empty((F, D, 2), dtype=F64, device=X.device)
    call("fmx_cs_moment_stats", CS[op], ptr(X), ptr(Y), F, D, A, A, ptr(present), ptr(stats), stream_ptr())
    return Y, stats


def cs_zscore_neutralize(X, out_z=None, out_n=None, present=None, with_stats=False):
    """cs_zscore and market_neutralize from one set of row moments (fmx_cs_zscore_neutralize).
    Returns (Yz, Yn) or (Yz, Yn, stats[F][D][2])."""
    X = as3(X)
    _check_panel(X)
    F, D, A = X.shape
    _check_present(present, D, A)
    Yz, Yn = _out(X, out_z), _out(X, out_n)
    stats = torch.empty((F, D, 2), dtype=F64, device=X.device) if with_stats else None
    call("fmx_cs_zscore_neutralize", ptr(X), ptr(Yz), ptr(Yn), F, D, A, A, ptr(present), ptr(stats), stream_ptr())
    return (Yz, Yn, stats) if with_stats else (Yz, Yn)


RANKED_IC_MAX_A = 16384
FINE_RANK_MAX_A = 16384     # fine-bucket rank / quantile kernels; longer rows are sorted in HBM
RANK2_DTYPE = torch.int16   # fmx_rank2_t: doubled ranks <= 2A as uint16 bit patterns
BITONIC_RANK_MAX_A = 8192   # fmx_cs_rank's LDS bitonic path (methods first / dense)
_WORK = {}


def _workspace(device, n):
    """Device scratch of >= n int32 words for the library calls that take a workspace
    (fmx_*_work_len / fmx_*_work_bytes): one buffer per (device, stream), grown on demand
    and reused, so the hot path never allocates.  Calls on one stream are ordered, so
    consecutive ops share it safely; another stream gets its own buffer."""
    key = (device, torch.cuda.current_stream(device).cuda_stream)
    w = _WORK.get(key)
    if w is None or w.numel() < n:
        w = torch.empty(max(n, 1), dtype=torch.int32, device=device)
        _WORK[key] = w
    return w


def _workspace_bytes(device, nbytes):
    n = (int(nbytes) + 3) // 4
    return _workspace(device, n), 4 * max(n, 1)


def cs_rank_winsor(X, qlo=0.01, qhi=0.99, out_rank=None, out_winsor=None, present=None, rank2=None):
    """cs_rank(average) and cs_winsor(qlo, qhi) in one pass (fmx_cs_rank_winsor).
    ``rank2`` (int16 tensor shaped like X, bit pattern uint16): also the doubled ranks that
    ``ic_daily(..., rank2=)`` starts from."""
    X = as3(X)
    _check_panel(X)
    F, D, A = X.shape
    _check_present(present, D, A)
    Yr, Yw = _out(X, out_rank), _out(X, out_winsor)
    if rank2 is not None:
        if rank2.dtype != RANK2_DTYPE or tuple(rank2.shape) != (F, D, A) or not rank2.is_contiguous():
            raise _lib.FmxError("rank2 must be a contiguous int16 (bit pattern uint16) [F][D][A] tensor")
    if A > FINE_RANK_MAX_A and rank2 is None:
        # rows past the fused kernel: both operators from rows sorted in HBM
        cs_rank(X, "average", present, out=Yr)
        cs_quantile_op("winsor", X, qlo, qhi, present, out=Yw)
        return Yr, Yw
    call("fmx_cs_rank_winsor", ptr(X), ptr(Yr), ptr(Yw), F, D, A, A, float(qlo), float(qhi), ptr(present),
         ptr(rank2), stream_ptr())
    return Yr, Yw


def cs_rank_winsor_zn(X, qlo=0.01, qhi=0.99, out_rank=None, out_winsor=None, out_zscore=None, out_neutralize=None,
                      rank2=None, dates=None):
    """cs_rank(average), cs_winsor(qlo, qhi), cs_zscore and market_neutralize of the same
    dense rows in one pass (fmx_cs_rank_winsor_zn: each row read once); every output is
    bit-identical to its own kernel.  ``rank2``: also the doubled ranks (as cs_rank_winsor).
    ``dates`` = (d0, d1): only the rows of those dates (fmx_cs_rank_winsor_zn_dates; the other
    rows of the outputs are left as they are; A <= 16384).
    Returns (Yrank, Ywinsor, Yzscore, Yneutralize)."""
    X = as3(X)
    _check_panel(X)
    F, D, A = X.shape
    outs = [_out(X, o) for o in (out_rank, out_winsor, out_zscore, out_neutralize)]
    if rank2 is not None:
        if rank2.dtype != RANK2_DTYPE or tuple(rank2.shape) != (F, D, A) or not rank2.is_contiguous():
            raise _lib.FmxError("rank2 must be a contiguous int16 (bit pattern uint16) [F][D][A] tensor")
    if dates is not None:
        d0, d1 = (int(d) for d in dates)
        call("fmx_cs_rank_winsor_zn_dates", ptr(X), *[ptr(o) for o in outs], F, D, A, A, d0, d1, float(qlo),
             float(qhi), ptr(rank2), stream_ptr())
        return tuple(outs)
    if A > FINE_RANK_MAX_A and rank2 is None:
        cs_rank_winsor(X, qlo, qhi, outs[0], outs[1])
        cs_zscore_neutralize(X, outs[2], outs[3])
        return tuple(outs)
    call("fmx_cs_rank_winsor_zn", ptr(X), *[ptr(o) for o in outs], F, D, A, A, float(qlo), float(qhi), ptr(rank2),
         stream_ptr())
    return tuple(outs)


def cs_rank_winsor_ic(X, R, lags=(1, 2), qlo=0.01, qhi=0.99, out_rank=None, out_winsor=None, ranks_only=False,
                      rank2=None):
    """cs_rank(average) + cs_winsor(qlo, qhi) and the daily IC records of the same rows in
    ONE pass (fmx_cs_rank_winsor_ic): returns (Yrank, Ywinsor, daily [L][4][F][D]);
    ``ranks_only``: no operator outputs (the IC's rank pass alone; Yrank = Ywinsor = None).
    ``rank2``: int16 [F][D][A] scratch for rows with long NaN-return lists (allocated when
    None).  Dense rows, A <= 16384, one or two lags."""
    X = as3(X)
    _check_panel(X)
    F, D, A = X.shape
    if tuple(R.shape) != (D, A) or R.dtype != F64 or not R.is_contiguous() or R.device != X.device:
        raise _lib.FmxError("R must be a contiguous float64 [D][A] tensor on X's device")
    if len(lags) not in (1, 2):
        raise _lib.FmxError("cs_rank_winsor_ic: one or two lags")
    Yr = Yw = None
    if not ranks_only:
        Yr, Yw = _out(X, out_rank), _out(X, out_winsor)
    if rank2 is None:
        rank2 = torch.empty((F, D, A), dtype=RANK2_DTYPE, device=X.device)
    elif rank2.dtype != RANK2_DTYPE or tuple(rank2.shape) != (F, D, A) or not rank2.is_contiguous():
        raise _lib.FmxError("rank2 must be a contiguous int16 [F][D][A] tensor")
    lag_h = (ctypes.c_int32 * len(lags))(*[int(v) for v in lags])
    n = int(_lib.load().fmx_rank_ic_work_len(F, D, A))
    work = _workspace(X.device, n)
    out = torch.empty((len(lags), 4, F, D), dtype=F64, device=X.device)
    call("fmx_cs_rank_winsor_ic", ptr(X), ptr(Yr), ptr(Yw), ptr(R), F, D, A, A, float(qlo), float(qhi),
         ctypes.cast(lag_h, ctypes.c_void_p), len(lags), ptr(rank2), ptr(work), n, ptr(out), stream_ptr())
    return Yr, Yw, out


def cs_rank2(X, rank2=None, dates=None):
    """Doubled average ranks only (fmx_cs_rank2): the rank pass ``ic_daily(..., rank2=)``
    starts from when no operator output of the rows is wanted (dense rows, A <= 16384).
    ``dates`` = (d0, d1): only the rows of those dates (fmx_cs_rank2_dates)."""
    X = as3(X)
    _check_panel(X)
    F, D, A = X.shape
    if rank2 is None:
        rank2 = torch.empty((F, D, A), dtype=RANK2_DTYPE, device=X.device)
    elif rank2.dtype != RANK2_DTYPE or tuple(rank2.shape) != (F, D, A) or not rank2.is_contiguous():
        raise _lib.FmxError("rank2 must be a contiguous int16 [F][D][A] tensor")
    if dates is not None:
        d0, d1 = (int(d) for d in dates)
        call("fmx_cs_rank2_dates", ptr(X), ptr(rank2), F, D, A, A, d0, d1, stream_ptr())
        return rank2
    call("fmx_cs_rank2", ptr(X), ptr(rank2), F, D, A, A, stream_ptr())
    return rank2


def cs_rank(X, method="average", present=None, out=None):
    X = as3(X)
    _check_panel(X)
    F, D, A = X.shape
    _check_present(present, D, A)
    if method not in RANK:
        raise ValueError(f"unknown rank method {method!r}")
    Y = _out(X, out)
    if (method in ("first", "dense") and A > BITONIC_RANK_MAX_A) or A > FINE_RANK_MAX_A:
        # rows past the LDS bitonic kernel (first / dense) or the fine-bucket kernels (the
        # other methods): sorted in HBM (fmx_cs_rank_sorted)
        nb = int(_lib.load().fmx_cs_rank_sorted_work_bytes(F, D, A))
        work, wb = _workspace_bytes(X.device, nb)
        call("fmx_cs_rank_sorted", ptr(X), ptr(Y), F, D, A, A, RANK[method], ptr(present), ptr(work), wb,
             stream_ptr())
        return Y
    call("fmx_cs_rank", ptr(X), ptr(Y), F, D, A, A, RANK[method], ptr(present), stream_ptr())
    return Y


def cs_quantile_op(kind: str, X, qlo: float, qhi: float, present=None, out=None):
    X = as3(X)
    _check_panel(X)
    F, D, A = X.shape
    _check_present(present, D, A)
    Y = _out(X, out)
    if A > FINE_RANK_MAX_A:
        # past the fine-bucket quantile kernels: order statistics of rows sorted in HBM
        nb = int(_lib.load().fmx_cs_rank_sorted_work_bytes(F, D, A))
        work, wb = _workspace_bytes(X.device, nb)
        call("fmx_cs_quantile_sorted", 0 if kind == "winsor" else 1, ptr(X), ptr(Y), F, D, A, A, float(qlo),
             float(qhi), ptr(present), ptr(work), wb, stream_ptr())
        return Y
    fn = "fmx_cs_winsor" if kind == "winsor" else "fmx_cs_filter_center"
    call(fn, ptr(X), ptr(Y), F, D, A, A, float(qlo), float(qhi), ptr(present), stream_ptr())
    return Y


def group_op(op: str, X, G, ngroups: int, method="average", present=None, long_rows=None):
    """Group ops (operations.py:104-168).  Rows past 16,384 assets (or ``long_rows=True``):
    rank from rows sorted by (group, value) in HBM, mean / neutralize / normalize with the
    members compacted in HBM scratch (fmx_group_op_long)."""
    X = as3(X)
    _check_panel(X)
    F, D, A = X.shape
    _check_present(present, D, A)
    if G.dtype != torch.int32 or tuple(G.shape) != (D, A):
        raise _lib.FmxError("G must be int32 [D][A]")
    if op == "rank" and A > 4096 and ngroups > 0:
        big = A > FINE_RANK_MAX_A
        if not big:
            # codes outside [0, ngroups) belong to no group (the kernel sorts them past the
            # last boundary); clamp the index so the count never writes out of bounds
            ok = (G >= 0) & (G < ngroups)
            if present is not None:
                ok &= present != 0
            cnt = torch.zeros((D, ngroups), dtype=torch.int32, device=G.device)
            cnt.scatter_add_(1, G.clamp(0, ngroups - 1).long(), ok.int())
            big = int(cnt.max()) > 8192          # the per-group LDS sort takes <= 8192 members
        if big:
            # rows sorted by (group, value) in HBM (fmx_group_rank_sorted): any group size
            Y = torch.empty_like(X)
            nb = int(_lib.load().fmx_group_rank_sorted_work_bytes(F, D, A))
            work, wb = _workspace_bytes(X.device, nb)
            call("fmx_group_rank_sorted", ptr(X), ptr(G), ptr(Y), F, D, A, A, int(ngroups), RANK[method],
                 ptr(present), ptr(work), wb, stream_ptr())
            return Y
    elif op != "rank" and (long_rows or (long_rows is None and A > FINE_RANK_MAX_A)):
        Y = torch.empty_like(X)
        nb = int(_lib.load().fmx_group_op_long_work_bytes(F, D, A))
        work, wb = _workspace_bytes(X.device, nb)
        call("fmx_group_op_long", GROUP[op], ptr(X), ptr(G), ptr(Y), F, D, A, A, int(ngroups), ptr(present),
             ptr(work), wb, stream_ptr())
        return Y
    Y = torch.empty_like(X)
    call("fmx_group_op", GROUP[op], ptr(X), ptr(G), ptr(Y), F, D, A, A, int(ngroups), RANK[method], ptr(present),
         stream_ptr())
    return Y


def cs_regression(Yv, Xv, rettype: str, present=None):
    D, A = Yv.shape
    if tuple(Xv.shape) != (D, A):
        raise _lib.FmxError("cs_regression: shape mismatch")
    _check_present(present, D, A)
    out = torch.empty_like(Yv)
    call("fmx_cs_regression", ptr(Yv), ptr(Xv), ptr(out), D, A, A, CSREG[rettype], ptr(present), stream_ptr())
    return out


def elementwise(op: str, X, a=0.0, b=0.0):
    X = X.contiguous()
    Y = torch.empty_like(X)
    call("fmx_elementwise", EW[op], ptr(X), ptr(Y), X.numel(), float(a), float(b), stream_ptr())
    return Y


def bucket_codes(X, edges: np.ndarray):
    X = X.contiguous()
    e = torch.as_tensor(np.asarray(edges, dtype=np.float64), device=X.device)
    codes = torch.empty(X.shape, dtype=torch.int32, device=X.device)
    call("fmx_bucket", ptr(X), ptr(codes), X.numel(), ptr(e), len(edges), stream_ptr())
    return codes


# ----------------------------------------------------------------------------- IC / selection
def ic_daily(X, R, lags=(1,), rank2=None, sorted_rows=None):
    """[n_lags][4][F][D] = (n_pairs, IC, rank_IC, beta) for pairs (X[f][t-L], R[t]).
    ``rank2``: the doubled ranks of X from ``cs_rank_winsor(X, rank2=...)`` -- the rows
    are then not ranked again (fmx_ic_daily_ranked, identical records).  Rows past 16,384
    assets (or ``sorted_rows=True``) are sorted in HBM (fmx_ic_daily_sorted)."""
    X = as3(X)
    _check_panel(X)
    F, D, A = X.shape
    if tuple(R.shape) != (D, A) or R.dtype != F64 or not R.is_contiguous():
        raise _lib.FmxError("R must be a contiguous float64 [D][A] device tensor")
    lag_h = (ctypes.c_int32 * len(lags))(*[int(v) for v in lags])
    out = torch.empty((len(lags), 4, F, D), dtype=F64, device=X.device)
    if rank2 is not None:
        if rank2.dtype != RANK2_DTYPE or tuple(rank2.shape) != (F, D, A) or not rank2.is_contiguous():
            raise _lib.FmxError("rank2 must be a contiguous int16 [F][D][A] tensor")
        n = int(_lib.load().fmx_ic_ranked_work_len(F, D))
        work = _workspace(X.device, n)
        call("fmx_ic_daily_ranked", ptr(X), ptr(rank2), ptr(R), F, D, A, A, ctypes.cast(lag_h, ctypes.c_void_p),
             len(lags), ptr(work), n, ptr(out), stream_ptr())
        return out
    if sorted_rows or (sorted_rows is None and A > RANKED_IC_MAX_A):
        # rows past the fine / LDS kernels: sorted in HBM, ranks read off the sorted rows
        nb = int(_lib.load().fmx_ic_daily_sorted_work_bytes(F, D, A))
        work, wb = _workspace_bytes(X.device, nb)
        call("fmx_ic_daily_sorted", ptr(X), ptr(R), F, D, A, A, ctypes.cast(lag_h, ctypes.c_void_p), len(lags),
             ptr(out), ptr(work), wb, stream_ptr())
        return out
    call("fmx_ic_daily", ptr(X), ptr(R), F, D, A, A, ctypes.cast(lag_h, ctypes.c_void_p), len(lags), ptr(out),
         stream_ptr())
    return out


def ic_window(daily, d0, d1):
    """daily [4][F][D]; windows [d0[j], d1[j]) -> [J][F][8]."""
    _, F, D = daily.shape
    daily = daily.contiguous()
    d0t = torch.as_tensor(np.asarray(d0, dtype=np.int32), device=daily.device)
    d1t = torch.as_tensor(np.asarray(d1, dtype=np.int32), device=daily.device)
    J = len(d0t)
    out = torch.empty((J, F, 8), dtype=F64, device=daily.device)
    call("fmx_ic_window", ptr(daily), F, D, ptr(d0t), ptr(d1t), J, ptr(out), stream_ptr())
    return out


def select_icir_top(metrics, use_rank_icir=True, threshold=0.03, top_x=5):
    J, F, _ = metrics.shape
    metrics = metrics.contiguous()
    order = torch.empty((J, F), dtype=torch.int32, device=metrics.device)
    w = torch.empty((J, F), dtype=F64, device=metrics.device)
    call("fmx_select_icir_top", ptr(metrics), J, F, int(bool(use_rank_icir)), float(threshold), int(top_x),
         ptr(order), ptr(w), stream_ptr())
    return order, w


def zscore_exposures(X, stats=None):
    """Z (per-date z-score, NaN -> 0, sigma in {0, NaN} -> row 0) and M (bf16 0/1) from
    the numpy-pairwise row moments of cs_moment_stats (the oracle's, bit for bit)."""
    X = as3(X)
    _check_panel(X)
    F, D, A = X.shape
    if stats is None:
        _, stats = cs_moment_stats("stats", X)
    Z = torch.empty_like(X)
    M = torch.empty(X.shape, dtype=torch.bfloat16, device=X.device)   # 0/1 validity
    call("fmx_zscore_exposures", ptr(X), ptr(stats), ptr(Z), ptr(M), F, D, A, A, stream_ptr())
    return Z, M


def gram(Z, M=None, d0=0, d1=None):
    F, D, A = Z.shape
    d1 = D if d1 is None else d1
    G = torch.empty((F, F), dtype=F64, device=Z.device)
    N = torch.empty((F, F), dtype=F64, device=Z.device) if M is not None else None
    nb = int(_lib.load().fmx_gram_work_bytes(F, D, A, int(d0), int(d1), int(M is not None)))
    work, wb = _workspace_bytes(Z.device, nb)
    call("fmx_gram", ptr(Z), ptr(M), ptr(G), ptr(N), F, D, A, A, int(d0), int(d1), 0, ptr(work), wb, stream_ptr())
    return G, N


FUSED_GRAM_MAX_F = 256


def gram_fused(X, stats, d0=0, d1=None):
    """G, N straight from the raw panel with row stats (F <= 256): one pass over X.
    ``stats=None``: X already holds the z-scores (the cs_zscore output of the rows)."""
    X = as3(X)
    _check_panel(X)
    F, D, A = X.shape
    if stats is not None and (tuple(stats.shape) != (F, D, 2) or stats.dtype != F64 or not stats.is_contiguous()):
        raise _lib.FmxError("stats must be a contiguous float64 [F][D][2] device tensor")
    d1 = D if d1 is None else d1
    G = torch.empty((F, F), dtype=F64, device=X.device)
    N = torch.empty((F, F), dtype=F64, device=X.device)
    nb = int(_lib.load().fmx_gram_fused_work_bytes(F, D, A, int(d0), int(d1)))
    work, wb = _workspace_bytes(X.device, nb)
    call("fmx_gram_fused", ptr(X), ptr(stats), ptr(G), ptr(N), F, D, A, A, int(d0), int(d1), 0, ptr(work), wb,
         stream_ptr())
    return G, N


GRAM_EXACT_SLOTS = 7            # fmx.h FMX_GRAM_EXACT_SLOTS: 6 payload limbs + flag


def gram_exact(X, stats=None, d0=0, d1=None, limbs=None, counts=None, accumulate=False):
    """Exact fixed-point Gram partials over dates [d0, d1) (fmx_gram_exact, F <= 256):
    (limbs int64 [7][F][F], counts int64 [F][F]), upper triangles.  Integer sums: ranks
    add them with any all-reduce and gram_exact_finalize gives the same G / N bits at every
    GPU count.  ``stats=None``: X holds the z-scores (the step's cs_zscore output)."""
    X = as3(X)
    _check_panel(X)
    F, D, A = X.shape
    if F > FUSED_GRAM_MAX_F:
        raise _lib.FmxError("gram_exact: F <= 256")
    if stats is not None and (tuple(stats.shape) != (F, D, 2) or stats.dtype != F64 or not stats.is_contiguous()):
        raise _lib.FmxError("stats must be a contiguous float64 [F][D][2] device tensor")
    d1 = D if d1 is None else d1
    if limbs is None:
        limbs = torch.empty((GRAM_EXACT_SLOTS, F, F), dtype=torch.int64, device=X.device)
    if counts is None:
        counts = torch.empty((F, F), dtype=torch.int64, device=X.device)
    if tuple(limbs.shape) != (GRAM_EXACT_SLOTS, F, F) or limbs.dtype != torch.int64 or not limbs.is_contiguous() \
            or tuple(counts.shape) != (F, F) or counts.dtype != torch.int64 or not counts.is_contiguous():
        raise _lib.FmxError("gram_exact: limbs int64 [7][F][F], counts int64 [F][F]")
    nb = int(_lib.load().fmx_gram_exact_work_bytes(F, D, A, int(d0), int(d1)))
    work, wb = _workspace_bytes(X.device, nb)
    call("fmx_gram_exact", ptr(X), ptr(stats), ptr(limbs), ptr(counts), F, D, A, A, int(d0), int(d1),
         int(bool(accumulate)), ptr(work), wb, stream_ptr())
    return limbs, counts


def gram_exact_finalize(limbs, counts):
    """G, N [F][F] float64 (symmetric) from (all-reduced) exact limbs / counts."""
    F = limbs.shape[1]
    G = torch.empty((F, F), dtype=F64, device=limbs.device)
    N = torch.empty((F, F), dtype=F64, device=limbs.device)
    call("fmx_gram_exact_finalize", ptr(limbs.contiguous()), ptr(counts.contiguous()), ptr(G), ptr(N), F,
         stream_ptr())
    return G, N


GRAM_CHUNK_BYTES = 8 << 30      # Z + M workspace of one date chunk of the wide Gram


def gram_chunked(X, d0=0, d1=None, chunk=None):
    """G, N over dates [d0, d1) for wide factor sets (F > 256, e.g. C4's 2000): Z / M are
    materialised one date chunk at a time (fmx_zscore_exposures_range, <= GRAM_CHUNK_BYTES)
    and accumulated into G / N by the tiled fp64 / bf16 MFMA kernels in chunk order
    (deterministic), so the panel never needs a full-size Z next to it."""
    X = as3(X)
    _check_panel(X)
    F, D, A = X.shape
    d1 = D if d1 is None else d1
    if chunk is None:
        chunk = max(1, min(d1 - d0, int(GRAM_CHUNK_BYTES // max(1, F * A * 10))))
    _, stats = cs_moment_stats("stats", X)
    G = torch.zeros((F, F), dtype=F64, device=X.device)
    N = torch.zeros((F, F), dtype=F64, device=X.device)
    Z = M = None
    for c0 in range(d0, d1, chunk):
        c1 = min(d1, c0 + chunk)
        n = c1 - c0
        if Z is None or Z.shape[1] != n:
            Z = torch.empty((F, n, A), dtype=F64, device=X.device)
            M = torch.empty((F, n, A), dtype=torch.bfloat16, device=X.device)
        call("fmx_zscore_exposures_range", ptr(X), ptr(stats), ptr(Z), ptr(M), F, D, A, A, c0, c1, stream_ptr())
        nb = int(_lib.load().fmx_gram_work_bytes(F, n, A, 0, n, 1))
        work, wb = _workspace_bytes(X.device, nb)
        call("fmx_gram", ptr(Z), ptr(M), ptr(G), ptr(N), F, n, A, A, 0, n, 1, ptr(work), wb, stream_ptr())
    return G, N


def gram_direct(X, d0=0, d1=None, stats=None):
    """G, N over dates [d0, d1) for wide factor sets (F > 256, C4's 2000) straight from
    the panel (fmx_gram_direct): the z-score (row stats of fmx_cs_moment_stats, computed
    here unless given) is applied while each tile chunk is staged and N comes from the
    validity bits on the i8 matrix cores -- no Z / M panels in HBM."""
    X = as3(X)
    _check_panel(X)
    F, D, A = X.shape
    d1 = D if d1 is None else d1
    if stats is None:
        _, stats = cs_moment_stats("stats", X)
    elif tuple(stats.shape) != (F, D, 2) or stats.dtype != F64 or not stats.is_contiguous():
        raise _lib.FmxError("stats must be a contiguous float64 [F][D][2] device tensor")
    G = torch.empty((F, F), dtype=F64, device=X.device)
    N = torch.empty((F, F), dtype=F64, device=X.device)
    nb = int(_lib.load().fmx_gram_direct_work_bytes(F, D, A, int(d0), int(d1)))
    work, wb = _workspace_bytes(X.device, nb)
    call("fmx_gram_direct", ptr(X), ptr(stats), ptr(G), ptr(N), F, D, A, A, int(d0), int(d1), 0, ptr(work), wb,
         stream_ptr())
    return G, N


GRAM_DATE_BLOCK = 16            # fmx.h FMX_GRAM_DATE_BLOCK: date shards align to it (wide Gram)


def gram_direct_exact(X, d0=0, d1=None, d_origin=0, stats=None, limbs=None, counts=None, accumulate=False):
    """Exact fixed-point partials of the wide Gram over dates [d0, d1) (fmx_gram_direct_exact,
    any F): (limbs int64 [7][F][F], counts int64 [F][F]).  Slices are absolute blocks of
    GRAM_DATE_BLOCK dates (local row 0 = absolute date ``d_origin``), so shards aligned to
    the block sum (int64 all-reduce) to the same bits at any GPU count; gram_exact_finalize
    gives G, N."""
    X = as3(X)
    _check_panel(X)
    F, D, A = X.shape
    d1 = D if d1 is None else d1
    if stats is None:
        pass            # the kernel's z pass (or, past its row size, its own stats pass) computes the moments
    elif tuple(stats.shape) != (F, D, 2) or stats.dtype != F64 or not stats.is_contiguous():
        raise _lib.FmxError("stats must be a contiguous float64 [F][D][2] device tensor")
    if limbs is None:
        limbs = torch.empty((GRAM_EXACT_SLOTS, F, F), dtype=torch.int64, device=X.device)
    if counts is None:
        counts = torch.empty((F, F), dtype=torch.int64, device=X.device)
    if tuple(limbs.shape) != (GRAM_EXACT_SLOTS, F, F) or limbs.dtype != torch.int64 or not limbs.is_contiguous() \
            or tuple(counts.shape) != (F, F) or counts.dtype != torch.int64 or not counts.is_contiguous():
        raise _lib.FmxError("gram_direct_exact: limbs int64 [7][F][F], counts int64 [F][F]")
    nb = int(_lib.load().fmx_gram_direct_exact_work_bytes(F, D, A, int(d0), int(d1), int(d_origin)))
    work, wb = _workspace_bytes(X.device, nb)
    call("fmx_gram_direct_exact", ptr(X), ptr(stats), ptr(limbs), ptr(counts), F, D, A, A, int(d0), int(d1),
         int(d_origin), int(bool(accumulate)), ptr(work), wb, stream_ptr())
    return limbs, counts


def gram_wide(X, d0=0, d1=None):
    """The wide (F > 256) Gram: direct from the panel by default; FMX_GRAM_MATERIALIZE=1
    selects the date-chunked Z / M path (A/B)."""
    import os
    if os.environ.get("FMX_GRAM_MATERIALIZE") == "1":
        return gram_chunked(X, d0, d1)
    return gram_direct(X, d0, d1)


def corr_matrix(X, d0=0, d1=None, stats=None):
    """Builder-defined factor correlation: C = G / N on fp64 MFMA.  F <= 256
    takes the fused path (row stats from cs_moment, one pass over X); wider panels
    materialise Z/M and use the 128x128-tiled kernels."""
    X = as3(X)
    if X.shape[0] <= FUSED_GRAM_MAX_F:
        if stats is None:
            _, stats = cs_moment_stats("stats", X)
        G, N = gram_fused(X, stats, d0, d1)
    else:
        G, N = gram_wide(X, d0, d1)
    return torch.where(N > 0, G / N.clamp_min(1.0), torch.zeros_like(G))


def corr_prune_windows(X, stats, metrics, order, window: int, s0, use_rank_icir=True, threshold=-np.inf, rho=0.7,
                       top_x=5):
    """Rolling corr_prune selection on the device (fmx_corr_prune_windows): weights [J][F]."""
    X = as3(X)
    _check_panel(X)
    F, D, A = X.shape
    J = metrics.shape[0]
    if tuple(metrics.shape) != (J, F, 8) or tuple(order.shape) != (J, F) or order.dtype != torch.int32:
        raise _lib.FmxError("corr_prune_windows: metrics [J][F][8] and int32 order [J][F] expected")
    s0h = (ctypes.c_int32 * J)(*[int(v) for v in s0])
    w = torch.empty((J, F), dtype=F64, device=X.device)
    top = F if top_x is None else int(top_x)
    s0p = ctypes.cast(s0h, ctypes.c_void_p)
    nb = int(_lib.load().fmx_corr_prune_windows_work_bytes(F, D, J, int(window), s0p))
    work, wb = _workspace_bytes(X.device, nb)
    call("fmx_corr_prune_windows", ptr(X), ptr(stats.contiguous()), F, D, A, A, J, int(window), s0p,
         ptr(order.contiguous()), ptr(metrics.contiguous()), int(bool(use_rank_icir)), float(threshold), float(rho),
         top, ptr(w), ptr(work), wb, stream_ptr())
    return w


def _greedy_prune_device(C, order, rho, top_x):
    if C.dim() != 2 or C.shape[0] != C.shape[1] or C.dtype != F64:
        raise _lib.FmxError("greedy_prune: C must be a square float64 matrix")
    C = C.contiguous()
    F = C.shape[0]
    if isinstance(order, torch.Tensor):
        ordt = order.to(device=C.device, dtype=torch.int64).contiguous()
    else:
        ordt = torch.as_tensor(np.asarray(order, dtype=np.int64), device=C.device)
    # the host walk returns once len(kept) >= top_x after an append: top_x <= 0 keeps one
    lim = F if top_x is None else max(int(top_x), 1)
    # the walk appends at most one entry per element of ``order`` (a repeated index can be kept
    # twice, as in the host walk): the bound handed to the kernel is also the buffer's capacity
    lim = min(lim, max(int(ordt.numel()), 1))
    kept = torch.empty(lim, dtype=torch.int32, device=C.device)
    nk = torch.zeros(1, dtype=torch.int32, device=C.device)
    call("fmx_greedy_prune", ptr(C), F, F, ptr(ordt), int(ordt.numel()), float(rho), lim, ptr(kept), ptr(nk),
         stream_ptr())
    n = int(nk.item())
    return [int(v) for v in kept[:n].cpu().tolist()]


def greedy_prune(C, order, rho=0.7, top_x=None):
    """Walk ``order``; keep f iff max |C[f, kept]| < rho (NaN: kept).  A device C runs the
    walk on the GPU (fmx_greedy_prune: no F x F copy to the host); a host C the numpy walk."""
    if isinstance(C, torch.Tensor) and C.is_cuda:
        return _greedy_prune_device(C, order, rho, top_x)
    Cn = C.detach().cpu().numpy() if isinstance(C, torch.Tensor) else np.asarray(C)
    # f is kept iff max_k |C[f, k]| over the kept k is < rho or NaN (np.max propagates NaN
    # and NaN >= rho is False).  Blocks of candidates: mx[g] = that max over the kept
    # columns of earlier blocks (np.maximum propagates NaN too); inside a block the walk is
    # sequential on the block's own |C| sub-matrix; then mx absorbs the block's kept columns.
    mx = np.full(Cn.shape[0], -np.inf)
    order = np.asarray(order, dtype=np.int64)
    kept = []
    B = 64
    for b0 in range(0, order.size, B):
        cand = order[b0:b0 + B]
        prior = mx[cand]
        sub = np.abs(Cn[np.ix_(cand, cand)])
        kin = []
        bm = np.full(cand.size, -np.inf)     # max over this block's kept columns so far
        for i in range(cand.size):
            p, m = prior[i], bm[i]
            if p == p and m == m and max(p, m) >= rho:
                continue                     # (a NaN among the kept columns keeps it)
            np.maximum(bm, sub[:, i], out=bm)
            kin.append(i)
            kept.append(int(cand[i]))
            if top_x is not None and len(kept) >= top_x:
                return kept
        if not kin:
            continue
        np.maximum(mx, np.abs(Cn[:, cand[kin]]).max(axis=1), out=mx)
    return kept


def device_info():
    buf = ctypes.create_string_buffer(256)
    call("fmx_device_info", buf, 256)
    return buf.value.decode()


# ----------------------------------------------------------------------------- composites
SUFFIXES = ["_eq", "_flx", "_long", "_short"]          # codes 1..4 (composite_factor.py:158-163)
_QLO = np.array([0, 10, 2, 2, 2], dtype=np.float64)
_QHI = np.array([0, 90, 98, 98, 98], dtype=np.float64)


def suffix_code(name: str) -> int:
    """composite_factor.py applies the suffix rules in this order; first match wins."""
    for k, s in enumerate(SUFFIXES):
        if name.endswith(s):
            return k + 1
    return 0


def _qfrac(dev):
    # np.nanpercentile(clean, [q_low, q_high]) divides integer percents by 100
    lo = torch.as_tensor(np.true_divide(_QLO, 100), device=dev)
    hi = torch.as_tensor(np.true_divide(_QHI, 100), device=dev)
    return lo, hi


def _i32(a, dev):
    return torch.as_tensor(np.ascontiguousarray(np.asarray(a, dtype=np.int32)), device=dev)


def comp_adj(X, cols, suffix_codes):
    _check_panel(X)
    F, D, A = X.shape
    K = len(cols)
    dev = X.device
    lo, hi = _qfrac(dev)
    c, s = _i32(cols, dev), _i32(suffix_codes, dev)
    Adj = torch.empty((K, D, A), dtype=F64, device=dev)
    call("fmx_comp_adj", ptr(X), ptr(c), ptr(s), ptr(lo), ptr(hi), ptr(Adj), K, D, A, stream_ptr())
    return Adj


def comp_proxy(Adj, groups):
    """groups: list of column-index lists into Adj."""
    K, D, A = Adj.shape
    dev = Adj.device
    gcols = _i32([c for g in groups for c in g], dev)
    goff = _i32(np.concatenate([[0], np.cumsum([len(g) for g in groups])]), dev)
    G = len(groups)
    P = torch.empty((G, D, A), dtype=F64, device=dev)
    call("fmx_comp_proxy", ptr(Adj), ptr(gcols), ptr(goff), ptr(P), G, D, A, stream_ptr())
    return P


def comp_combine(Nrm, mode, present=None):
    G, D, A = Nrm.shape
    out = torch.empty((D, A), dtype=F64, device=Nrm.device)
    call("fmx_comp_combine", ptr(Nrm), G, D, A, int(mode), ptr(present), ptr(out), stream_ptr())
    return out


def wcomp(X, plan, method, present=None):
    """weighted_composite_factor device stages for a host-built ``plan`` (see
    composite_factor._weighted_plan).  Returns the [D][A] composite (0 where unselected)."""
    _check_panel(X)
    F, D, A = X.shape
    dev = X.device
    J = len(plan["pdate"])
    out = torch.zeros((D, A), dtype=F64, device=dev)
    if J == 0:
        return out
    KMAX = plan["KMAX"]
    pdate, ncol = _i32(plan["pdate"], dev), _i32(plan["ncol"], dev)
    col, suf, grp = _i32(plan["col"], dev), _i32(plan["suf"], dev), _i32(plan["grp"], dev)
    soff, scol = _i32(plan["soff"], dev), _i32(plan["scol"], dev)
    ngrp = _i32(plan["ngrp"], dev)
    gw = torch.as_tensor(plan["gw"], device=dev)
    lo, hi = _qfrac(dev)
    lohi = torch.empty((J, 4, 3), dtype=F64, device=dev)
    call("fmx_wcomp_pct", ptr(X), ptr(pdate), ptr(soff), ptr(scol), J, D, A, ptr(lo), ptr(hi), ptr(lohi),
         stream_ptr())
    G = max(1, int(plan["ngrp"].max()))
    P = torch.empty((G, J, A), dtype=F64, device=dev)
    call("fmx_wcomp_proxy", ptr(X), ptr(pdate), ptr(ncol), ptr(col), ptr(suf), ptr(grp), KMAX, J, D, A, ptr(lohi), G,
         ptr(P), stream_ptr())
    presJ = None
    if present is not None:
        pd_idx = torch.as_tensor(np.maximum(plan["pdate"], 0), device=dev, dtype=torch.long)
        presJ = present[pd_idx].contiguous()
        P.masked_fill_(presJ.unsqueeze(0) == 0, float("nan"))
    if method == "zscore":
        Nrm = cs_moment("market_neutralize", P, presJ)
    else:
        Nrm = cs_rank(P, "scipy_average", presJ)
    call("fmx_wcomp_combine", ptr(Nrm), ptr(pdate), ptr(ngrp), ptr(gw), KMAX, J, D, A, ptr(present), ptr(out),
         stream_ptr())
    return out


# ----------------------------------------------------------------------------- trade list
def trade_equal(X, pct: float, present=None):
    """Simulation._daily_trade_list, method 'equal' (portfolio_simulation.py:96-170) on one
    [D][A] signal panel: (per-symbol shift(1) of the day's weights [D][A], counts [D][2])."""
    if X.dim() != 2 or X.dtype != F64 or not X.is_cuda:
        raise _lib.FmxError("X must be a float64 [D][A] device tensor")
    X = X.contiguous()
    D, A = X.shape
    _check_present(present, D, A)
    Wraw = torch.empty_like(X)
    Wout = torch.empty_like(X)
    counts = torch.empty((D, 2), dtype=F64, device=X.device)
    call("fmx_trade_equal", ptr(X), ptr(present), ptr(Wraw), ptr(Wout), ptr(counts), D, A, float(pct),
         stream_ptr())
    return Wout, counts


def trade_linear(X, max_weight: float, present=None):
    """Simulation._daily_trade_list, method 'linear' (portfolio_simulation.py:172-181,
    :250-313) on one [D][A] panel: (shifted weights [D][A], counts [D][2])."""
    if X.dim() != 2 or X.dtype != F64 or not X.is_cuda:
        raise _lib.FmxError("X must be a float64 [D][A] device tensor")
    X = X.contiguous()
    D, A = X.shape
    _check_present(present, D, A)
    Wraw, Wout = torch.empty_like(X), torch.empty_like(X)
    counts = torch.empty((D, 2), dtype=F64, device=X.device)
    call("fmx_trade_linear", ptr(X), ptr(present), ptr(Wraw), ptr(Wout), ptr(counts), D, A, float(max_weight),
         stream_ptr())
    return Wout, counts


TRADE_METHODS = {"equal": 0, "linear": 1}


def trade_books(X, method: str, pct=0.1, max_weight=0.03, present=None, nan_absent=True, raw=False):
    """F trade books in one launch (fmx_trade_books): X [F][D][A] -> (shifted [F][D][A],
    counts [F][D][2]) (+ the same-day books with ``raw``); with nan_absent a NaN cell is no row."""
    X = as3(X)
    _check_panel(X)
    F, D, A = X.shape
    _check_present(present, D, A)
    if method not in TRADE_METHODS:
        raise NotImplementedError(f"method {method!r}: the device runs 'equal' and 'linear'")
    Wraw, Wout = torch.empty_like(X), torch.empty_like(X)
    counts = torch.empty((F, D, 2), dtype=F64, device=X.device)
    call("fmx_trade_books", TRADE_METHODS[method], ptr(X), ptr(present), int(bool(nan_absent)), ptr(Wraw),
         ptr(Wout), ptr(counts), F, D, A, float(pct), float(max_weight), stream_ptr())
    return (Wout, counts, Wraw) if raw else (Wout, counts)


def shift_rows(W):
    """Per-symbol shift(1) over each book's present (non-NaN) rows (fmx_shift_rows)."""
    W = as3(W).contiguous()
    F, D, A = W.shape
    out = torch.empty_like(W)
    call("fmx_shift_rows", ptr(W), ptr(out), F, D, A, stream_ptr())
    return out


def mm_combine(Wf, counts, fw, colmap, wdate):
    """multi_manager combination (multi_manager.py:51-72) of fmx_trade_equal outputs."""
    F, D, A = Wf.shape
    Dw, Fw = fw.shape
    if tuple(counts.shape) != (F, D, 2) or len(colmap) != Fw or len(wdate) != Dw:
        raise _lib.FmxError("mm_combine: shape mismatch")
    cm = np.asarray(colmap, dtype=np.int32)
    wd = np.asarray(wdate, dtype=np.int32)
    if (cm >= F).any() or (wd >= D).any():
        raise _lib.FmxError("mm_combine: colmap/wdate out of range")
    dev = Wf.device
    fw_d = torch.as_tensor(np.ascontiguousarray(fw, dtype=np.float64), device=dev)
    cm_d = torch.as_tensor(cm, device=dev)
    wd_d = torch.as_tensor(wd, device=dev)
    out = torch.empty((Dw, A), dtype=F64, device=dev)
    oc = torch.empty((Dw, 2), dtype=F64, device=dev)
    call("fmx_mm_combine", ptr(Wf.contiguous()), ptr(counts.contiguous()), ptr(fw_d), ptr(cm_d), ptr(wd_d),
         ptr(out), ptr(oc), Fw, Dw, D, A, stream_ptr())
    return out, oc


# ----------------------------------------------------------------------------- P&L
def _dense2(X, name):
    if X.dim() != 2 or X.dtype != F64 or not X.is_cuda or not X.is_contiguous():
        raise _lib.FmxError(f"{name} must be a contiguous float64 [D][A] device tensor")


def pnl_daily(W, R, CAP, wprev, contrib=False):
    """Simulation._daily_portfolio_returns per-date sums (fmx_pnl_daily): [D][6] and the
    optional per-symbol [A][2] contributions."""
    _dense2(W, "W")
    _dense2(R, "R")
    D, A = W.shape
    if tuple(R.shape) != (D, A) or (CAP is not None and (tuple(CAP.shape) != (D, A))):
        raise _lib.FmxError("pnl_daily: shape mismatch")
    if CAP is not None:
        _dense2(CAP, "CAP")
    wp = torch.as_tensor(np.ascontiguousarray(np.asarray(wprev, dtype=np.int32)), device=W.device)
    if wp.numel() != D or (wp >= D).any():
        raise _lib.FmxError("pnl_daily: wprev must be [D] row indices < D (or -1)")
    out = torch.empty((D, 6), dtype=F64, device=W.device)
    cb = torch.empty((A, 2), dtype=F64, device=W.device) if contrib else None
    call("fmx_pnl_daily", ptr(W), ptr(R), ptr(CAP), ptr(wp), ptr(out), ptr(cb), D, A, stream_ptr())
    return out, cb


def daily_corr(X, R):
    """Per-date Pearson (np.corrcoef) of pair-valid cells (fmx_daily_corr): [D][2] = (n, corr)."""
    _dense2(X, "X")
    _dense2(R, "R")
    D, A = X.shape
    if tuple(R.shape) != (D, A):
        raise _lib.FmxError("daily_corr: shape mismatch")
    out = torch.empty((D, 2), dtype=F64, device=X.device)
    call("fmx_daily_corr", ptr(X), ptr(R), ptr(out), D, A, stream_ptr())
    return out
