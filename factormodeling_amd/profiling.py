"""Opt-in wall-clock breakdown of the drop-in API's host <-> device boundary (VERDICT r5
item 6; SURVEY 8(d): the pandas <-> dense conversion and the H2D / D2H copies are reported
apart from the kernels).  Off by default: ``phase()`` is then a no-op.  When enabled, each
phase synchronises the device on entry and exit, so its time is exactly that step; what is
left of a call's wall time is the device work (kernel launches + kernels) and Python glue.

    with profiling.record() as ph:
        single_factor_metrics(df, ret)
    ph  ->  {"pandas->dense": s, "H2D": s, "D2H": s, "dense->pandas": s}
"""
from __future__ import annotations

import contextlib
import time
from collections import defaultdict

import torch

_acc = None
_depth = 0


@contextlib.contextmanager
def phase(name):
    global _depth
    if _acc is None or _depth:                 # disabled, or inside another phase
        yield
        return
    _depth += 1
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    try:
        yield
    finally:
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        _acc[name] += time.perf_counter() - t0
        _depth -= 1


@contextlib.contextmanager
def record():
    """Enable the phase timers for the enclosed calls; yields the dict they fill."""
    global _acc
    prev = _acc
    _acc = defaultdict(float)
    out = _acc
    try:
        yield out
    finally:
        _acc = prev
