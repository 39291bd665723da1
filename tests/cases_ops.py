"""Operator case table shared by the oracle-vs-golden and GPU-vs-golden tests.

Each case: key -> (oracle(x, y, g, present) -> dense[D][A],
                   api(ops_module, sx, sy, sg) -> pd.Series,
                   exact)   # True: bit-exact required (ranks, pandas-emulated kernels)
"""
from __future__ import annotations

import oracle.ops as O


def _c(fn_o, fn_api, exact=True):
    return (fn_o, fn_api, exact)


CASES = {}
for w in (3, 5, 20):
    CASES[f"ts_sum_{w}"] = _c(lambda x, y, g, p, w=w: O.ts_sum(x, w, p), lambda m, x, y, g, w=w: m.ts_sum(x, w))
    CASES[f"ts_mean_{w}"] = _c(lambda x, y, g, p, w=w: O.ts_mean(x, w, p), lambda m, x, y, g, w=w: m.ts_mean(x, w))
    CASES[f"ts_std_{w}"] = _c(lambda x, y, g, p, w=w: O.ts_std(x, w, p), lambda m, x, y, g, w=w: m.ts_std(x, w))
    CASES[f"ts_zscore_{w}"] = _c(lambda x, y, g, p, w=w: O.ts_zscore(x, w, p), lambda m, x, y, g, w=w: m.ts_zscore(x, w))
    CASES[f"ts_rank_{w}"] = _c(lambda x, y, g, p, w=w: O.ts_rank(x, w, p), lambda m, x, y, g, w=w: m.ts_rank(x, w))
    CASES[f"ts_diff_{w}"] = _c(lambda x, y, g, p, w=w: O.ts_diff(x, w, p), lambda m, x, y, g, w=w: m.ts_diff(x, w))
    CASES[f"ts_delay_{w}"] = _c(lambda x, y, g, p, w=w: O.ts_delay(x, w, p), lambda m, x, y, g, w=w: m.ts_delay(x, w))
    CASES[f"ts_decay_{w}"] = _c(lambda x, y, g, p, w=w: O.ts_decay(x, w, p), lambda m, x, y, g, w=w: m.ts_decay(x, w), False)
CASES["ts_decay_0"] = _c(lambda x, y, g, p: O.ts_decay(x, 0, p), lambda m, x, y, g: m.ts_decay(x, 0))
CASES["ts_decay_1"] = _c(lambda x, y, g, p: O.ts_decay(x, 1, p), lambda m, x, y, g: m.ts_decay(x, 1), False)
CASES["ts_backfill"] = _c(lambda x, y, g, p: O.ts_backfill(x, p), lambda m, x, y, g: m.ts_backfill(x))
for meth in ("average", "min", "max", "first", "dense"):
    CASES[f"cs_rank_{meth}"] = _c(lambda x, y, g, p, meth=meth: O.cs_rank(x, p, meth),
                                  lambda m, x, y, g, meth=meth: m.cs_rank(x, method=meth))
CASES["cs_winsor"] = _c(lambda x, y, g, p: O.cs_winsor(x, p), lambda m, x, y, g: m.cs_winsor(x))
CASES["cs_winsor_10_90"] = _c(lambda x, y, g, p: O.cs_winsor(x, p, (0.1, 0.9)),
                              lambda m, x, y, g: m.cs_winsor(x, limits=(0.1, 0.9)))
CASES["cs_filter_center"] = _c(lambda x, y, g, p: O.cs_filter_center(x, p), lambda m, x, y, g: m.cs_filter_center(x))
CASES["cs_filter_center_20_60"] = _c(lambda x, y, g, p: O.cs_filter_center(x, p, (0.2, 0.6)),
                                     lambda m, x, y, g: m.cs_filter_center(x, center=(0.2, 0.6)))
CASES["cs_zscore"] = _c(lambda x, y, g, p: O.cs_zscore(x, p), lambda m, x, y, g: m.cs_zscore(x))
CASES["cs_mean"] = _c(lambda x, y, g, p: O.cs_mean(x, p), lambda m, x, y, g: m.cs_mean(x))
CASES["market_neutralize"] = _c(lambda x, y, g, p: O.market_neutralize(x, p), lambda m, x, y, g: m.market_neutralize(x))
CASES["cs_bool"] = _c(lambda x, y, g, p: O.cs_bool(x > 0, 1.0, -1.0), lambda m, x, y, g: m.cs_bool(x > 0, 1.0, -1.0))
CASES["sign"] = _c(lambda x, y, g, p: O.sign(x), lambda m, x, y, g: m.sign(x))
CASES["power_2"] = _c(lambda x, y, g, p: O.power(x, 2), lambda m, x, y, g: m.power(x, 2))
CASES["power_0.5"] = _c(lambda x, y, g, p: O.power(x, 0.5), lambda m, x, y, g: m.power(x, 0.5), False)
CASES["log"] = _c(lambda x, y, g, p: O.log(x), lambda m, x, y, g: m.log(x), False)
CASES["abs"] = _c(lambda x, y, g, p: O.abs_(x), lambda m, x, y, g: m.abs_(x))
CASES["clip"] = _c(lambda x, y, g, p: O.clip(x, -0.5, 0.5), lambda m, x, y, g: m.clip(x, -0.5, 0.5))
CASES["group_mean"] = _c(lambda x, y, g, p: O.group_mean(x, g, p), lambda m, x, y, g: m.group_mean(x, g))
CASES["group_neutralize"] = _c(lambda x, y, g, p: O.group_neutralize(x, g, p), lambda m, x, y, g: m.group_neutralize(x, g))
CASES["group_normalize"] = _c(lambda x, y, g, p: O.group_normalize(x, g, p), lambda m, x, y, g: m.group_normalize(x, g))
CASES["group_rank_normalized"] = _c(lambda x, y, g, p: O.group_rank_normalized(x, g, p),
                                    lambda m, x, y, g: m.group_rank_normalized(x, g))
for rt in ("resid", "beta", "alpha", "fitted", "r2"):
    CASES[f"cs_regression_{rt}"] = _c(lambda x, y, g, p, rt=rt: O.cs_regression(y, x, p, rt),
                                      lambda m, x, y, g, rt=rt: m.cs_regression(y, x, rettype=rt))

# ts_regression_fast has a row-subset output index: handled separately
TSREG = [(lag, rt) for lag in (0, 1) for rt in (0, 1, 2, 3, 6)]
BUCKETS = [(0.2, 1.0, 0.2), (0.0, 1.0, 0.25)]
