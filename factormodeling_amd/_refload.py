"""Loader for the reference's own HOST-ONLY modules (outside the GPU scope):
the MVO trade-list solvers (portfolio_simulation.py:183-248, :315-746) and
``mvo_selector`` (factor_selection_methods.py:119-175), both cvxpy / scipy QPs per date.

They are loaded by file path from ``$FMX_REFERENCE_DIR`` under a private module name.
The directory is on ``sys.path`` only while the module body executes (its top-level
``from portfolio_analyzer import ...``), then removed again, so no later import can
resolve the reference's other top-level modules (operations, factor_selector, ...)
instead of the drop-ins.  No hot-path function calls this module
(tests/test_refload.py).
"""
from __future__ import annotations

import importlib.util
import os
import sys

_CACHE: dict = {}


def reference_dir(what: str) -> str:
    d = os.environ.get("FMX_REFERENCE_DIR")
    if not d or not os.path.isdir(d):
        raise NotImplementedError(f"{what} runs the reference's host QP solvers: set FMX_REFERENCE_DIR to the "
                                  "FactorModeling checkout that holds the reference modules")
    return d


def load(filename: str, what: str):
    """The reference module ``filename`` (e.g. 'portfolio_simulation.py'), cached."""
    d = reference_dir(what)
    path = os.path.join(d, filename)
    if not os.path.exists(path):
        raise NotImplementedError(f"{what}: {path} not found (FMX_REFERENCE_DIR)")
    key = os.path.realpath(path)
    if key in _CACHE:
        return _CACHE[key]
    name = "_fmx_reference_" + os.path.splitext(filename)[0]
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    added = d not in sys.path
    if added:
        sys.path.insert(0, d)
    try:
        spec.loader.exec_module(mod)
    finally:
        if added:
            try:
                sys.path.remove(d)
            except ValueError:
                pass
    _CACHE[key] = mod
    return mod
