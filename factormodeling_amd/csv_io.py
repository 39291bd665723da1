"""Native long-CSV loader: the data step in front of the factor-panel path.

Reference counterpart (pipeline.ipynb:71-82)::

    factors_df = pd.read_csv('data/8.factors_df.csv')
    factors_df['date'] = pd.to_datetime(factors_df['date'])
    factors_df.set_index(['date', 'symbol'], inplace=True)

``read_long_csv(path)`` returns the same DataFrame (same index order, level dtypes, column
order, float64 values bit-identical to pandas' default C parser, int64 for all-integer
columns); ``symbol_col=None`` covers the date-indexed wide file
(9.single_factor_returns.csv).  ``load_panel(path)`` skips pandas entirely and returns the
engine's dense ``[F][D][A]`` panel (NaN where a (date, symbol) row is absent), optionally
straight into HBM through a pinned staging buffer.

Parsing runs in libfmx_io.so (csrc/csv_io.cpp, C ABI in include/fmx_io.h) on host
threads.  There is no pandas fallback: a missing library or an unsupported file (quoted
fields, non-ISO dates, non-numeric values) raises.
"""
from __future__ import annotations

import ctypes
import os
import re
from dataclasses import dataclass

import numpy as np
import pandas as pd

from .panel import PanelIndex

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FMX_IO_LIB", os.path.join(_HERE, "libfmx_io.so"))

c_i32, c_i64, c_vp, c_cp = ctypes.c_int32, ctypes.c_int64, ctypes.c_void_p, ctypes.c_char_p
_P64 = ctypes.POINTER(c_i64)
_P32 = ctypes.POINTER(c_i32)

SIGNATURES = {
    "fmx_io_last_error": [],
    "fmx_parse_double": [c_cp, c_i64, ctypes.POINTER(ctypes.c_double)],
    "fmx_csv_open": [c_cp, c_cp, c_cp, c_i32, ctypes.POINTER(c_vp)],
    "fmx_csv_close": [c_vp],
    "fmx_csv_shape": [c_vp, _P64, _P64, _P64, _P64, _P32],
    "fmx_csv_strings": [c_vp, c_i32, c_vp, c_i64, _P64],
    "fmx_csv_dates": [c_vp, c_vp],
    "fmx_csv_rows": [c_vp, c_vp],
    "fmx_csv_int_columns": [c_vp, c_vp],
    "fmx_csv_values": [c_vp, c_vp, c_i32],
    "fmx_csv_dense": [c_vp, c_vp, c_i32],
    "fmx_csv_write": [c_cp, c_cp, c_cp, c_cp, c_vp, c_i64, c_i64, c_i64, c_vp, c_i32],
    "fmx_format_double": [ctypes.c_double, c_vp, c_i32],
}

_lib = None


class FmxIOError(RuntimeError):
    pass


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FmxIOError(f"{LIB_PATH} not built (run `make -C factormodeling_amd/csrc`)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, args in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = c_cp if name == "fmx_io_last_error" else c_i32
        _lib = lib
    return _lib


def _check(rc):
    if rc != 0:
        raise FmxIOError(load().fmx_io_last_error().decode())


def parse_double(s: str) -> float | None:
    """pandas' default float parser on one field (None if pandas would not parse it)."""
    b = s.encode()
    out = ctypes.c_double()
    return out.value if load().fmx_parse_double(b, len(b), ctypes.byref(out)) else None


def format_double(x: float) -> str:
    """repr(float) as the writer emits it ('' for NaN, pandas' na_rep)."""
    buf = ctypes.create_string_buffer(64)
    n = load().fmx_format_double(float(x), buf, 64)
    return buf.raw[:n].decode() if n > 0 else ""


class _Csv:
    def __init__(self, path, date_col, symbol_col, threads):
        self.lib = load()
        self.h = c_vp()
        _check(self.lib.fmx_csv_open(os.fsencode(path), date_col.encode(),
                                     (symbol_col or "").encode(), int(threads or 0), ctypes.byref(self.h)))
        n, F, D, A = (c_i64() for _ in range(4))
        srt = c_i32()
        _check(self.lib.fmx_csv_shape(self.h, *(ctypes.byref(x) for x in (n, F, D, A, srt))))
        self.n, self.F, self.D, self.A = n.value, F.value, D.value, A.value
        self.per_symbol_sorted = bool(srt.value)
        self.threads = int(threads or 0)

    def strings(self, which):
        need = c_i64()
        _check(self.lib.fmx_csv_strings(self.h, which, None, 0, ctypes.byref(need)))
        buf = ctypes.create_string_buffer(max(1, need.value))
        _check(self.lib.fmx_csv_strings(self.h, which, buf, need.value, ctypes.byref(need)))
        return buf.raw[:need.value].decode().split("\n")[:-1]

    def arr(self, fn, shape, dtype, *extra):
        a = np.empty(shape, dtype=dtype)
        _check(getattr(self.lib, fn)(self.h, a.ctypes.data_as(c_vp), *extra))
        return a

    def close(self):
        if self.h:
            self.lib.fmx_csv_close(self.h)
            self.h = c_vp()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


_INT_RE = re.compile(r"^\s*[+-]?\d{1,18}\s*$")


def _symbol_level(syms):
    """pandas parses an all-integer symbol column as int64; mirror that."""
    if syms and all(_INT_RE.match(s) for s in syms):
        return pd.Index(np.array([int(s) for s in syms], dtype=np.int64))
    return pd.Index(syms, dtype=object)


@dataclass
class Panel:
    dates: pd.DatetimeIndex
    symbols: pd.Index
    names: list
    X: object  # np.ndarray or torch.Tensor [F][D][A] float64
    per_symbol_sorted: bool


def load_panel(path, date_col="date", symbol_col="symbol", threads=None, device=None) -> Panel:
    """Dense ``[F][D][A]`` panel of a long CSV (dates and symbols sorted, NaN where absent).

    ``device`` (e.g. ``"cuda:0"``): the panel is written into a pinned host tensor and
    copied to HBM; otherwise a numpy array is returned."""
    with _Csv(path, date_col, symbol_col, threads) as c:
        names = c.strings(0)
        syms = c.strings(1) if symbol_col else [""]
        dates = pd.DatetimeIndex(c.arr("fmx_csv_dates", c.D, np.int64).view("datetime64[ns]"), name=date_col)
        shape = (c.F, c.D, c.A)
        if device is not None:
            import torch
            host = torch.empty(shape, dtype=torch.float64, pin_memory=torch.cuda.is_available())
            _check(c.lib.fmx_csv_dense(c.h, c_vp(host.data_ptr()), c.threads))
            X = host.to(device, non_blocking=True)
        else:
            X = c.arr("fmx_csv_dense", shape, np.float64, c.threads)
        level = _symbol_level(syms) if symbol_col else pd.Index(syms)
        if symbol_col and level.dtype != object:
            order = np.argsort(level.values, kind="stable")
            if not np.array_equal(order, np.arange(len(order))):
                X = X[:, :, order] if isinstance(X, np.ndarray) else X[:, :, order.tolist()].contiguous()
                level = level[order]
        return Panel(dates, level.rename(symbol_col), names, X, c.per_symbol_sorted)


def read_long_csv(path, date_col="date", symbol_col="symbol", threads=None) -> pd.DataFrame:
    """``pd.read_csv`` + ``pd.to_datetime(date)`` + ``set_index([date, symbol])`` of the
    reference notebook (pipeline.ipynb:71-82), parsed natively.  ``symbol_col=None``:
    index by date only (pipeline.ipynb:79-82)."""
    with _Csv(path, date_col, symbol_col, threads) as c:
        names = c.strings(0)
        syms = c.strings(1) if symbol_col else None
        dts = c.arr("fmx_csv_dates", c.D, np.int64).view("datetime64[ns]")
        flat = c.arr("fmx_csv_rows", c.n, np.int64)
        vals = c.arr("fmx_csv_values", (c.n, c.F), np.float64, c.threads)
        ints = c.arr("fmx_csv_int_columns", c.F, np.int32)
    A = max(len(syms), 1) if syms is not None else 1
    d_of_row = flat // A
    date_vals = pd.DatetimeIndex(dts[d_of_row], name=date_col)
    if symbol_col:
        level = _symbol_level(syms)
        sym_vals = level.take(flat % A)
        index = pd.MultiIndex.from_arrays([date_vals, sym_vals], names=[date_col, symbol_col])
    else:
        index = date_vals
    cols = {}
    for j, name in enumerate(names):
        col = vals[:, j]
        cols[name] = col.astype(np.int64) if ints[j] else col
    return pd.DataFrame(cols, index=index, columns=pd.Index(names, dtype=object))


def _plain(names, what):
    for n in names:
        if any(c in str(n) for c in ',"\n\r'):
            raise ValueError(f"{what} {n!r} would need CSV quoting; not supported by the native writer")
    return [str(n) for n in names]


def write_long_csv(obj, path, threads=None) -> None:
    """``obj.to_csv(path)`` for the notebook's checkpoint objects (pipeline.ipynb:217,364,
    391,420,464-466), byte-identical: a float64 DataFrame/Series indexed by a lexsorted
    ``(date, symbol)`` MultiIndex (factors, composite factor) or by dates (factor weights).
    Raises ValueError for anything else (no silent pandas fallback)."""
    frame = obj.to_frame() if isinstance(obj, pd.Series) else obj
    if isinstance(obj, pd.Series) and obj.name is None:
        frame.columns = ["0"]
    if not all(dt == np.float64 for dt in frame.dtypes):
        raise ValueError("native writer handles float64 columns only")
    cols = _plain(frame.columns, "column")
    idx = frame.index
    if isinstance(idx, pd.MultiIndex):
        if idx.nlevels != 2:
            raise ValueError("expected a (date, symbol) MultiIndex")
        pi = PanelIndex(idx)
        if np.any(np.diff(pi.flat) <= 0):
            raise ValueError("rows are not in (date, symbol) order")
        dates, syms = pi.dates, _plain(pi.symbols, "symbol")
        D, A = pi.D, pi.A
        X = pi.to_dense(frame.to_numpy(dtype=np.float64))
        present = None if pi.dense else np.ascontiguousarray(pi.present_np)
        names = [str(n) if n is not None else "" for n in idx.names]
    else:
        if idx.has_duplicates or not idx.is_monotonic_increasing:
            raise ValueError("index must be unique and increasing")
        dates, syms = idx, None
        D, A = len(idx), 1
        X = np.ascontiguousarray(frame.to_numpy(dtype=np.float64).T).reshape(len(cols), D, 1)
        present = None
        names = [str(idx.name) if idx.name is not None else ""]
    # D date strings formatted by pandas itself (same format decision as to_csv's)
    dstr = pd.Series(dates).to_csv(index=False, header=False).splitlines() if D else []
    if not isinstance(dates, pd.DatetimeIndex):
        dstr = _plain(dstr, "index value")
    header = ",".join(names + cols)
    X = np.ascontiguousarray(X, dtype=np.float64)
    _check(load().fmx_csv_write(os.fsencode(path), header.encode(), "".join(d + "\n" for d in dstr).encode(),
                                None if syms is None else "".join(s + "\n" for s in syms).encode(),
                                X.ctypes.data_as(c_vp), X.shape[0], D, A,
                                None if present is None else present.ctypes.data_as(c_vp), int(threads or 0)))
