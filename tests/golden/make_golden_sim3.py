"""Golden vectors for ``Simulation._daily_portfolio_returns``' contributor lists when the
returns and the cap flags cover DIFFERENT extra symbols (portfolio_simulation.py:792-795),
by running the REFERENCE in this container (test infrastructure only):

    python tests/golden/make_golden_sim3.py      -> tests/golden/sim3.npz

The reference subtracts a Series over weights ∪ returns symbols from one over weights ∪
cap_flag symbols, so a symbol found in only one of them aligns to NaN and ``nlargest``
drops it.  Extra symbols sort FIRST ("A…") so a zero in their place would win ties.
Plain arrays only (no pickles).
"""
from __future__ import annotations

import os
import sys
import warnings

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import OUT, import_reference, put_series  # noqa: E402


def main():
    warnings.filterwarnings("ignore")
    import_reference()
    import portfolio_simulation as ps
    rng = np.random.default_rng(91)
    st = {}
    cases = [("split_eq", 12, 8, "equal", 0.25), ("split_lin", 14, 10, "linear", 0.3)]
    for name, D, A, method, pct in cases:
        dates = pd.bdate_range("2021-06-01", periods=D)
        syms = [f"S{k:03d}" for k in range(A)]
        ret_syms = syms + ["AR00", "AR01", "ZR00"]           # returns-only symbols
        cap_syms = syms[1:] + ["AC00", "ZC00"]               # cap-only symbols; S000 has no cap flag
        sig = pd.Series(rng.standard_normal(D * A),
                        index=pd.MultiIndex.from_product([dates, syms], names=["date", "symbol"]))
        ridx = pd.MultiIndex.from_product([dates, ret_syms], names=["date", "symbol"])
        ret = pd.Series(0.01 * rng.standard_normal(len(ridx)), index=ridx)
        cidx = pd.MultiIndex.from_product([dates, cap_syms], names=["date", "symbol"])
        cap = pd.Series(rng.integers(1, 4, len(cidx)).astype(np.float64), index=cidx)
        inv = pd.Series(1.0, index=ret.index)
        union = sorted(set(syms) | set(ret_syms) | set(cap_syms))
        for tc in (True, False):
            settings = ps.SimulationSettings(returns=ret, cap_flag=cap, investability_flag=inv, factors_df=None,
                                             method=method, pct=pct, max_weight=0.5, plot=False,
                                             transaction_cost=tc, contributor=True)
            sim = ps.Simulation(name="g", custom_feature=sig, settings=settings)
            w, _ = sim._daily_trade_list()
            _, tl, tsh = sim._daily_portfolio_returns(w)
            key = f"{name}_tc{int(tc)}"
            st[f"{key}_top_long_s"] = np.array(list(tl.index))
            st[f"{key}_top_long_v"] = tl.to_numpy(dtype=np.float64)
            st[f"{key}_top_short_s"] = np.array(list(tsh.index))
            st[f"{key}_top_short_v"] = tsh.to_numpy(dtype=np.float64)
            if tc:
                st[f"{name}_syms"] = np.array(union)
                st[f"{name}_dates"] = np.array([str(d.date()) for d in dates])
                put_series(st, f"{name}_w", w, dates, union)
                put_series(st, f"{name}_ret", ret, dates, union)
                put_series(st, f"{name}_cap", cap, dates, union)
    np.savez_compressed(os.path.join(OUT, "sim3.npz"), **st)
    print("wrote sim3.npz:", len(st), "arrays")


if __name__ == "__main__":
    main()
