"""ctypes binding of libfmx.so (the HIP/gfx950 kernels behind the drop-in API).

There is no CPU fallback: if the shared library or a GPU is missing, every compute
entry point raises :class:`FmxError`.  ``torch`` is imported first so that the HIP
runtime torch ships with (``libamdhip64.so.7``) is the one libfmx binds to -- device
pointers and streams are then shared between torch and libfmx.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must be loaded before libfmx: one HIP runtime per process)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FMX_LIB", os.path.join(_HERE, "libfmx.so"))

c_i32, c_i64, c_dbl, c_vp, c_cp = ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p, ctypes.c_char_p

# name -> argtypes (restype is c_int32 = fmx_status unless listed in _RESTYPES)
SIGNATURES = {
    "fmx_last_error": [],
    "fmx_abi_version": [],
    "fmx_build_variant": [],
    "fmx_device_info": [c_cp, c_i64],
    "fmx_ts_op": [c_i32, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i32, c_vp, c_vp],
    "fmx_ts_set": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i32, c_i32, c_vp, c_vp],
    "fmx_ts_corr": [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_vp, c_vp],
    "fmx_ts_corr_vol_feature": [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i32, c_vp],
    "fmx_ts_corr_feature": [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_vp],
    "fmx_ts_regression": [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i32, c_i32, c_vp],
    "fmx_cs_moment": [c_i32, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp],
    "fmx_cs_moment_stats": [c_i32, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp],
    "fmx_cs_zscore_neutralize": [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp],
    "fmx_cs_rank_winsor": [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_dbl, c_dbl, c_vp, c_vp, c_vp],
    "fmx_cs_rank_winsor_zn": [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_dbl, c_dbl, c_vp, c_vp],
    "fmx_cs_rank_sorted": [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i32, c_vp, c_vp, c_i64, c_vp],
    "fmx_cs_rank_sorted_work_bytes": [c_i64, c_i64, c_i64],
    "fmx_cs_quantile_sorted": [c_i32, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_dbl, c_dbl, c_vp, c_vp, c_i64, c_vp],
    "fmx_group_rank_sorted": [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i32, c_i32, c_vp, c_vp, c_i64, c_vp],
    "fmx_group_rank_sorted_work_bytes": [c_i64, c_i64, c_i64],
    "fmx_cs_rank2": [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp],
    "fmx_cs_rank_winsor_zn_dates": [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_dbl,
                                    c_dbl, c_vp, c_vp],
    "fmx_cs_rank2_dates": [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp],
    "fmx_cs_rank": [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i32, c_vp, c_vp],
    "fmx_cs_winsor": [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_dbl, c_dbl, c_vp, c_vp],
    "fmx_cs_filter_center": [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_dbl, c_dbl, c_vp, c_vp],
    "fmx_group_op": [c_i32, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i32, c_i32, c_vp, c_vp],
    "fmx_cs_regression": [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i32, c_vp, c_vp],
    "fmx_elementwise": [c_i32, c_vp, c_vp, c_i64, c_dbl, c_dbl, c_vp],
    "fmx_bucket": [c_vp, c_vp, c_i64, c_vp, c_i32, c_vp],
    "fmx_ic_daily": [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_i32, c_vp, c_vp],
    "fmx_ic_ranked_work_len": [c_i64, c_i64],
    "fmx_ic_daily_ranked": [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_i32, c_vp, c_i64, c_vp, c_vp],
    "fmx_rank_ic_work_len": [c_i64, c_i64, c_i64],
    "fmx_cs_rank_winsor_ic": [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_dbl, c_dbl, c_vp, c_i32, c_vp, c_vp,
                              c_i64, c_vp, c_vp],
    "fmx_ic_window": [c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp],
    "fmx_select_icir_top": [c_vp, c_i64, c_i64, c_i32, c_dbl, c_i32, c_vp, c_vp, c_vp],
    "fmx_zscore_exposures": [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp],
    "fmx_corr_prune_windows": [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_vp, c_vp, c_vp, c_i32,
                               c_dbl, c_dbl, c_i32, c_vp, c_vp, c_i64, c_vp],
    "fmx_corr_prune_windows_work_bytes": [c_i64, c_i64, c_i64, c_i32, c_vp],
    "fmx_zscore_exposures_range": [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp],
    "fmx_gram": [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_vp, c_i64, c_vp],
    "fmx_gram_work_bytes": [c_i64, c_i64, c_i64, c_i64, c_i64, c_i32],
    "fmx_gram_direct": [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_vp, c_i64, c_vp],
    "fmx_gram_direct_work_bytes": [c_i64, c_i64, c_i64, c_i64, c_i64],
    "fmx_greedy_prune": [c_vp, c_i64, c_i64, c_vp, c_i64, c_dbl, c_i64, c_vp, c_vp, c_vp],
    "fmx_gram_direct_exact": [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_vp,
                              c_i64, c_vp],
    "fmx_gram_direct_exact_work_bytes": [c_i64, c_i64, c_i64, c_i64, c_i64, c_i64],
    "fmx_ic_daily_sorted": [c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_i32, c_vp, c_vp, c_i64, c_vp],
    "fmx_ic_daily_sorted_work_bytes": [c_i64, c_i64, c_i64],
    "fmx_group_op_long": [c_i32, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i32, c_vp, c_vp, c_i64, c_vp],
    "fmx_group_op_long_work_bytes": [c_i64, c_i64, c_i64],
    "fmx_gram_fused": [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_vp, c_i64, c_vp],
    "fmx_gram_fused_work_bytes": [c_i64, c_i64, c_i64, c_i64, c_i64],
    "fmx_gram_exact": [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_i32, c_vp, c_i64, c_vp],
    "fmx_gram_exact_work_bytes": [c_i64, c_i64, c_i64, c_i64, c_i64],
    "fmx_gram_exact_finalize": [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp],
    "fmx_gram_exact_units_per_date": [c_i64],
    "fmx_debug_exact_fold": [c_vp, c_i64, c_vp, c_vp],
    "fmx_debug_pw_schedule": [c_i32, c_vp, c_i32],
    "fmx_comp_adj": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp],
    "fmx_comp_proxy": [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp],
    "fmx_comp_combine": [c_vp, c_i64, c_i64, c_i64, c_i32, c_vp, c_vp, c_vp],
    "fmx_wcomp_pct": [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp],
    "fmx_wcomp_proxy": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i64, c_i64, c_i64, c_vp, c_i64, c_vp, c_vp],
    "fmx_trade_equal": [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_dbl, c_vp],
    "fmx_trade_linear": [c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_dbl, c_vp],
    "fmx_trade_books": [c_i32, c_vp, c_vp, c_i32, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_dbl, c_dbl, c_vp],
    "fmx_shift_rows": [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp],
    "fmx_mm_combine": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp],
    "fmx_pnl_daily": [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp],
    "fmx_daily_corr": [c_vp, c_vp, c_vp, c_i64, c_i64, c_vp],
    "fmx_wcomp_combine": [c_vp, c_vp, c_vp, c_vp, c_i32, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp],
}
_RESTYPES = {"fmx_last_error": c_cp, "fmx_build_variant": c_cp, "fmx_ic_ranked_work_len": c_i64, "fmx_rank_ic_work_len": c_i64, "fmx_gram_work_bytes": c_i64, "fmx_gram_direct_work_bytes": c_i64,
             "fmx_gram_direct_exact_work_bytes": c_i64, "fmx_ic_daily_sorted_work_bytes": c_i64,
             "fmx_group_op_long_work_bytes": c_i64,
             "fmx_gram_fused_work_bytes": c_i64, "fmx_corr_prune_windows_work_bytes": c_i64,
             "fmx_cs_rank_sorted_work_bytes": c_i64, "fmx_group_rank_sorted_work_bytes": c_i64, "fmx_gram_exact_work_bytes": c_i64,
             "fmx_debug_exact_fold": None}

# constants mirrored from include/fmx.h
TS = dict(sum=0, mean=1, std=2, var=3, zscore=4, rank=5, decay=6, diff=7, delay=8, backfill=9)
CS = dict(zscore=0, mean=1, market_neutralize=2, stats=3)
RANK = dict(average=0, min=1, max=2, first=3, dense=4, scipy_average=5)
GROUP = dict(mean=0, neutralize=1, normalize=2, rank=3)
EW = dict(sign=0, power=1, log=2, abs=3, clip=4, where=5)
CSREG = dict(resid=0, beta=1, alpha=2, fitted=3, r2=4)


class FmxError(RuntimeError):
    pass


_lib = None
_lock = threading.Lock()


def load(path: str = None):
    """Load libfmx.so (no GPU needed) and bind every exported entry point."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise FmxError(f"libfmx.so not found at {p}; build it with __graft_entry__.build() "
                           f"(make -C factormodeling_amd/csrc)")
        lib = ctypes.CDLL(p)
        for name, args in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = _RESTYPES.get(name, c_i32)
        variant = lib.fmx_build_variant().decode()
        if variant != "product" and os.environ.get("FMX_ALLOW_DIAG") != "1":
            raise FmxError(f"{p} is a {variant} build (wrong-result timing arms); "
                           f"set FMX_ALLOW_DIAG=1 to load it for A/B timing")
        if path is None:
            _lib = lib
        return lib


def require_gpu():
    if not torch.cuda.is_available():
        raise FmxError("factormodeling_amd needs an MI355X (HIP device); none is visible. "
                       "There is no CPU fallback by design.")


def call(name: str, *args):
    """Invoke an fmx_* entry point and raise FmxError on a non-zero status."""
    lib = load()
    st = getattr(lib, name)(*args)
    if st != 0:
        msg = lib.fmx_last_error()
        raise FmxError(f"{name} failed (status {st}): {msg.decode() if msg else ''}")


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def ptr(t):
    """Device pointer of a torch tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())
