"""Time the long-CSV loading step: reference pandas path vs libfmx_io.

    python tools/csv_bench.py --dates 252 --assets 2000 --factors 20 [--threads 8]

Writes a synthetic long file with pandas' to_csv (SURVEY 8(d) generator shape: 1% NaN,
5% 1-decimal values), then times
  ref     pd.read_csv + pd.to_datetime + set_index (pipeline.ipynb:71-82), 1 thread
  frame   csv_io.read_long_csv (same DataFrame)
  panel   csv_io.load_panel    (dense [F][D][A] numpy, what the engine uploads)
and checks frame == ref exactly.  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from factormodeling_amd import csv_io  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dates", type=int, default=252)
    ap.add_argument("--assets", type=int, default=2000)
    ap.add_argument("--factors", type=int, default=20)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--dir", default=tempfile.gettempdir())
    a = ap.parse_args()
    D, A, F = a.dates, a.assets, a.factors
    rng = np.random.default_rng(0)
    idx = pd.MultiIndex.from_product([pd.bdate_range("2015-01-01", periods=D),
                                      [f"S{k:05d}" for k in range(A)]], names=["date", "symbol"])
    X = rng.standard_normal((D * A, F))
    X[rng.random(X.shape) < 0.01] = np.nan
    X = np.where(rng.random(X.shape) < 0.05, np.round(X, 1), X)
    path = os.path.join(a.dir, f"fmx_csv_bench_{D}x{A}x{F}.csv")
    pd.DataFrame(X, index=idx, columns=[f"f{k:04d}" for k in range(F)]).to_csv(path)
    size = os.path.getsize(path)
    units = D * A * F

    t0 = time.perf_counter()
    ref = pd.read_csv(path)
    ref["date"] = pd.to_datetime(ref["date"])
    ref.set_index(["date", "symbol"], inplace=True)
    t_ref = time.perf_counter() - t0

    t0 = time.perf_counter()
    got = csv_io.read_long_csv(path, threads=a.threads)
    t_frame = time.perf_counter() - t0
    pd.testing.assert_frame_equal(got, ref, check_exact=True)

    t0 = time.perf_counter()
    pan = csv_io.load_panel(path, threads=a.threads)
    t_panel = time.perf_counter() - t0
    assert np.array_equal(pan.X.reshape(F, -1).T, ref.to_numpy(), equal_nan=True)
    t0 = time.perf_counter()
    ref.to_csv(path + ".ref")
    t_wref = time.perf_counter() - t0
    t0 = time.perf_counter()
    csv_io.write_long_csv(ref, path + ".got", threads=a.threads)
    t_write = time.perf_counter() - t0
    assert open(path + ".got", "rb").read() == open(path + ".ref", "rb").read()
    for q in (path, path + ".ref", path + ".got"):
        os.remove(q)
    print(json.dumps({"file_mb": round(size / 2**20, 1), "dims": [D, A, F], "threads": a.threads,
                      "ref_s": round(t_ref, 3), "frame_s": round(t_frame, 3), "panel_s": round(t_panel, 3),
                      "ref_units_per_s": units / t_ref, "panel_units_per_s": units / t_panel,
                      "panel_MBps": size / 2**20 / t_panel, "speedup_panel": t_ref / t_panel,
                      "write_ref_s": round(t_wref, 3), "write_s": round(t_write, 3),
                      "speedup_write": t_wref / t_write}))


if __name__ == "__main__":
    main()
