"""Adapter between the reference's long ``(date, symbol)`` MultiIndex objects and the
engine's dense ``[F][D][A]`` device panels.

The reference operates on pandas objects indexed by a ``(date, symbol)`` MultiIndex
(operations.py, factor_selector.py, composite_factor.py).  Its semantics are row-based:
``groupby(level='symbol')`` + ``rolling``/``shift`` walk each symbol's rows in input
order, and ``groupby(level='date')`` reduces over the rows of a date.  The adapter maps
every row to a cell of a dense ``dates x symbols`` grid (dates and symbols sorted) and
records which cells exist (``present``); the kernels then skip absent cells, which is
exactly row-based semantics as long as each symbol's rows appear in date order.  That
precondition is checked; inputs violating it raise ``ValueError``.
"""
from __future__ import annotations

import numpy as np
import pandas as pd
import torch

from .profiling import phase

F64 = torch.float64


class PanelIndex:
    def __init__(self, index: pd.MultiIndex):
        if not isinstance(index, pd.MultiIndex) or index.nlevels != 2:
            raise ValueError("expected a (date, symbol) MultiIndex")
        names = list(index.names)
        dl = index.get_level_values("date" if "date" in names else 0)
        sl = index.get_level_values("symbol" if "symbol" in names else 1)
        dcode, dates = pd.factorize(dl, sort=True)
        scode, syms = pd.factorize(sl, sort=True)
        if (dcode < 0).any() or (scode < 0).any():
            raise ValueError("NaN dates or symbols in the index are not supported")
        self.index = index
        self.dates = pd.Index(dates)
        self.symbols = pd.Index(syms)
        self.D, self.A = len(dates), len(syms)
        self.n = len(index)
        self.d = dcode.astype(np.int64)
        self.s = scode.astype(np.int64)
        self.flat = self.d * self.A + self.s
        if np.unique(self.flat).size != self.n:
            raise ValueError("duplicate (date, symbol) rows are not supported")
        self.dense = self.n == self.D * self.A and bool(np.all(self.flat == np.arange(self.n)))
        if not self.dense:
            order = np.lexsort((np.arange(self.n), self.s))
            dd = self.d[order]
            ss = self.s[order]
            same = ss[1:] == ss[:-1]
            if np.any(same & (dd[1:] <= dd[:-1])):
                raise ValueError("rows of a symbol are not in date order; the reference's row-based "
                                 "rolling windows would differ from calendar order (sort the index)")
            pres = np.zeros(self.D * self.A, dtype=np.uint8)
            pres[self.flat] = 1
            self.present_np = pres.reshape(self.D, self.A)
        else:
            self.present_np = None
        self._present_dev = {}

    def row_layout(self):
        """(pos, width, sorted_within): every row's position inside its date in INPUT order
        (the order a ``groupby('date')`` group presents its rows), the widest date, and
        whether that order is the sorted-symbol order on every date.  Per-date reductions
        whose rounding depends on row order (numpy pairwise sums) run on this layout."""
        order = np.argsort(self.d, kind="stable")
        dd = self.d[order]
        starts = np.searchsorted(dd, np.arange(self.D))
        pos = np.empty(self.n, dtype=np.int64)
        pos[order] = np.arange(self.n) - starts[dd]
        width = int(np.bincount(self.d, minlength=self.D).max()) if self.n else 0
        ss = self.s[order]
        same = dd[1:] == dd[:-1]
        sorted_within = not bool(np.any(same & (ss[1:] <= ss[:-1])))
        return pos, width, sorted_within

    # ------------------------------------------------------------------ host <-> dense
    def to_dense(self, values: np.ndarray) -> np.ndarray:
        """values [n] or [n][F] (row order) -> dense [F][D][A] (NaN where absent)."""
        v = np.asarray(values, dtype=np.float64)
        if v.ndim == 1:
            v = v[:, None]
        F = v.shape[1]
        if self.dense:
            return np.ascontiguousarray(v.T).reshape(F, self.D, self.A)
        out = np.full((F, self.D * self.A), np.nan)
        out[:, self.flat] = v.T
        return out.reshape(F, self.D, self.A)

    def gather(self, dense: np.ndarray) -> np.ndarray:
        """dense [F][D][A] -> [n][F] in row order."""
        F = dense.shape[0]
        flat = dense.reshape(F, self.D * self.A)
        if self.dense:
            return flat.T
        return flat[:, self.flat].T

    # ------------------------------------------------------------------ device
    def present(self, device):
        if self.present_np is None:
            return None
        key = str(device)
        if key not in self._present_dev:
            self._present_dev[key] = torch.as_tensor(self.present_np, device=device)
        return self._present_dev[key]

    def _flat_dev(self, device):
        key = ("flat", str(device))
        if key not in self._present_dev:
            self._present_dev[key] = torch.as_tensor(self.flat, device=device)
        return self._present_dev[key]

    def to_device(self, values, device) -> torch.Tensor:
        """values [n] or [n][F] (row order) -> device [F][D][A] (NaN where absent), as
        to_dense but with the transpose / scatter done on the device: the rows go up in
        whichever of the two orders the host array already has (a DataFrame's float block
        is [F][n] in memory; a host-side transpose of a C1 frame took ~90 ms, its H2D copy
        ~3 ms)."""
        with phase("pandas->dense"):
            v = np.asarray(values, dtype=np.float64)
            if v.ndim == 1:
                v = v[:, None]
            F = v.shape[1]
            fmajor = v.T.flags.c_contiguous             # the [F][n] layout in memory
            host = v.T if fmajor else np.ascontiguousarray(v)
        with phase("H2D"):
            t = torch.as_tensor(host, device=device)
        t = t if fmajor else t.T                        # [F][n] view
        if self.dense:
            return t.contiguous().reshape(F, self.D, self.A)
        out = torch.full((F, self.D * self.A), float("nan"), dtype=F64, device=device)
        out[:, self._flat_dev(device)] = t
        return out.reshape(F, self.D, self.A)

    def from_device(self, Y: torch.Tensor) -> np.ndarray:
        """device [F][D][A] -> host [n][F] in row order (gather): the gather and the
        transpose on the device, one D2H copy of the result."""
        F = Y.shape[0]
        flat = Y.detach().reshape(F, self.D * self.A)
        if not self.dense:
            flat = flat[:, self._flat_dev(Y.device)]
        rows = flat.T.contiguous() if F > 1 else flat.reshape(-1, 1)
        with phase("D2H"):
            return rows.cpu().numpy()


_CACHE: list = []


def panel_index(index: pd.MultiIndex) -> PanelIndex:
    """PanelIndex for ``index`` (cached by object identity; indexes are immutable)."""
    for idx, p in _CACHE:
        if idx is index:
            return p
    with phase("pandas->dense"):
        p = PanelIndex(index)
    _CACHE.append((index, p))
    del _CACHE[:-8]
    return p


def device():
    from . import _lib
    _lib.require_gpu()
    return torch.device("cuda", torch.cuda.current_device())
