"""Golden vectors for LONG rolling windows (the notebook's ts_decay sweep and hand-offs).

Test infrastructure only.  Run in the build container (where /root/reference exists):

    python tests/golden/make_golden_longwin.py

Imports the reference exactly as make_golden.py does and writes ``ops_longwin.npz``:
the reference operators (operations.py:6-51) on a 420-date panel, dense and ragged, at
the windows the notebook uses -- ``ts_decay`` at 80 / 150 (the Simulation hand-offs,
pipeline.ipynb:268,310,510) and 175 / 350 (the decay sweep reaches 350,
pipeline.ipynb:132,145) -- plus ``ts_rank`` at 60 / 200, the rolling moments and shifts
at 175 / 350, leads (negative windows) of 200, and the builder-defined ``ts_corr``
(pandas ``Rolling.corr``, no reference counterpart) and ``ts_regression_fast`` at 175.

The panel keeps NaNs sparse (one cell, one short run, one column-long gap) so that long
windows still produce values; half the cells of four columns are rounded to one decimal
(ties for ts_rank).  The ragged variant drops ~12 % of rows, lists one symbol late and
delists another early.
"""
from __future__ import annotations

import json
import os
import sys
import warnings

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import import_reference, put_series  # noqa: E402

D, A = 420, 12
DECAY_W = (80, 150, 175, 350)
RANK_W = (60, 200)
MOMENT_W = (175, 350)
LEAD = 200


def panel(rng, ragged):
    dates = pd.bdate_range("2016-01-01", periods=D)
    syms = [f"L{i:02d}" for i in range(A)]
    x = rng.standard_normal((D, A)) + 0.2 * np.arange(A)[None, :]
    tie = (rng.random((D, A)) < 0.5) & (np.arange(A)[None, :] % 3 == 0)
    x[tie] = np.round(x[tie], 1)
    x[130, 1] = np.nan                              # a single NaN
    x[240:246, 2] = np.nan                          # a short NaN run
    x[50:230, 5] = 0.25                             # a long constant run (ts_std exact 0)
    x[300, 7] = -0.0                                # a signed zero
    y = 0.4 * np.nan_to_num(x) + rng.standard_normal((D, A))
    y[rng.random((D, A)) < 0.01] = np.nan
    present = np.ones((D, A), dtype=bool)
    if ragged:
        present &= rng.random((D, A)) > 0.12
        present[:150, 3] = False                    # lists late
        present[300:, 4] = False                    # delists early
        present[:, 0] = True
    di, si = np.nonzero(present)
    idx = pd.MultiIndex.from_arrays([dates[di], [syms[k] for k in si]], names=["date", "symbol"])
    return dates, syms, pd.Series(x[di, si], index=idx, name="fx"), pd.Series(y[di, si], index=idx, name="fy")


def gen(ref_ops, rng, ragged):
    dates, syms, x, y = panel(rng, ragged)
    st = {"dates": np.array([str(d.date()) for d in dates]), "syms": np.array(syms)}
    put_series(st, "in_x", x, dates, syms)
    put_series(st, "in_y", y, dates, syms)
    cases = []

    def add(key, ser):
        put_series(st, "out_" + key, ser, dates, syms)
        cases.append(key)

    for w in DECAY_W:
        add(f"ts_decay_{w}", ref_ops.ts_decay(x, w))
    for w in RANK_W:
        add(f"ts_rank_{w}", ref_ops.ts_rank(x, w))
    for w in MOMENT_W:
        add(f"ts_sum_{w}", ref_ops.ts_sum(x, w))
        add(f"ts_mean_{w}", ref_ops.ts_mean(x, w))
        add(f"ts_std_{w}", ref_ops.ts_std(x, w))
        add(f"ts_zscore_{w}", ref_ops.ts_zscore(x, w))
        add(f"ts_diff_{w}", ref_ops.ts_diff(x, w))
        add(f"ts_delay_{w}", ref_ops.ts_delay(x, w))
    add(f"ts_diff_m{LEAD}", ref_ops.ts_diff(x, -LEAD))
    add(f"ts_delay_m{LEAD}", ref_ops.ts_delay(x, -LEAD))
    parts = [xs.rolling(175).corr(y.xs(sym, level="symbol", drop_level=False))
             for sym, xs in x.groupby(level="symbol")]
    add("ts_corr_175", pd.concat(parts).reindex(x.index))
    for rt in (0, 2):
        add(f"ts_regression_fast_175_1_{rt}", ref_ops.ts_regression_fast(y, x, 175, lag=1, rettype=rt))
    return st, cases


def main():
    warnings.filterwarnings("ignore")
    os.environ["TQDM_DISABLE"] = "1"
    ref_ops, _, _, _ = import_reference()
    path = os.path.join(HERE, "manifest.json")
    manifest = json.load(open(path))
    out = {}
    for tag, seed, ragged in (("dense", 700, False), ("ragged", 701, True)):
        st, cases = gen(ref_ops, np.random.default_rng(seed), ragged)
        out.update({f"{tag}/{k}": v for k, v in st.items()})
        manifest["files"].setdefault("ops_longwin.npz", {"generator": "make_golden_longwin.py", "D": D, "A": A})
        manifest["files"]["ops_longwin.npz"][tag] = {"seed": seed, "ragged": ragged, "cases": cases}
    np.savez_compressed(os.path.join(HERE, "ops_longwin.npz"), **out)
    with open(path, "w") as f:
        json.dump(manifest, f, indent=1)
    print("wrote ops_longwin.npz")


if __name__ == "__main__":
    main()
