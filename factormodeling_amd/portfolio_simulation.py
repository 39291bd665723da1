"""Drop-in replacement for the reference's ``portfolio_simulation.py`` (SURVEY §8(f) ranks
2 and 4).

``SimulationSettings`` and ``Simulation`` keep the reference's fields, defaults,
constructor and ``run()`` flow (portfolio_simulation.py:10-95).  The per-date work runs on
the GPU through libfmx:

* ``_daily_trade_list`` (:96-154): methods 'equal' (``k_trade_equal``, :156-170) and
  'linear' (``k_trade_linear``: normalised legs + cap-and-redistribute, :172-181,
  :250-313), then the per-symbol ``shift(1)``;
* ``_daily_portfolio_returns`` (:748-797): long / short P&L, turnover and the cap-flag
  transaction cost per date (``k_pnl_daily``) and the per-symbol contributions
  (``k_pnl_contrib``);
* ``_calculate_metrics`` (:799-819): the daily IC (``k_daily_corr``).

The MVO methods ('mvo', 'mvo_turnover', :183-248, :315-746) solve a cvxpy / scipy QP per
date on the host and stay the reference's own code: ``_daily_trade_list`` hands them to the
reference's ``Simulation``, loaded by file path from ``FMX_REFERENCE_DIR`` (the user's
reference checkout; a module of the same name cannot sit on ``sys.path`` next to this
drop-in), while the P&L and metrics of the resulting weights still run on the device.
``PortfolioAnalyzer`` (reporting and plots) is the reference's own host module, imported
from ``portfolio_analyzer`` when ``run()`` needs it.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import pandas as pd
import torch

from . import _refload
from . import engine as E
from .panel import device
from .simulation import daily_trade_list

RESULT_COLS = ["log_return", "long_return", "short_return", "long_turnover", "short_turnover", "turnover"]


@dataclass
class SimulationSettings:
    # market data
    returns: pd.Series             # MultiIndex (date, symbol)
    cap_flag: pd.Series            # MultiIndex (date, symbol)
    investability_flag: pd.Series  # MultiIndex (date, symbol)
    factors_df: pd.DataFrame       # your factor DataFrame
    # simulation parameters (with defaults)
    method: str = 'equal'          # 'equal' | 'linear' | 'mvo' | 'mvo_turnover'
    transaction_cost: bool = True
    max_weight: float = 0.03
    pct: float = 0.1
    min_universe: int = 1000
    contributor: bool = False
    output_summary: bool = False
    output_returns: bool = False
    plot: bool = True
    # MVO-specific parameters
    lookback_period: int = 60
    use_cvxpy: bool = True
    mvo_solver: str = 'OSQP'
    shrinkage_intensity: float = 0.1
    turnover_penalty: float = 0.1
    return_weight: float = 0.0


def reference_simulation_classes():
    """(Simulation, SimulationSettings) of the reference's ``portfolio_simulation.py``,
    loaded by path from ``$FMX_REFERENCE_DIR`` under a private module name (cached;
    ``_refload``: the directory is on ``sys.path`` only while the module body runs)."""
    mod = _refload.load("portfolio_simulation.py", "methods 'mvo' / 'mvo_turnover'")
    return mod.Simulation, mod.SimulationSettings


class _Grid:
    """Union (date, symbol) grid of several long Series: sorted unique dates and symbols
    (what ``unstack`` + frame alignment produce), and each Series as a dense [D][A]
    float64 array (NaN where it has no row)."""

    def __init__(self, *series):
        idx = [s.index for s in series if s is not None]
        self.dates = pd.Index(np.unique(np.concatenate([i.get_level_values(0).values for i in idx])))
        self.symbols = pd.Index(np.unique(np.concatenate([np.asarray(i.get_level_values(1), dtype=object)
                                                          for i in idx])))
        self.D, self.A = len(self.dates), len(self.symbols)

    def dense(self, s):
        out = np.full((self.D, self.A), np.nan)
        if s is not None and len(s):
            d = self.dates.get_indexer(s.index.get_level_values(0))
            a = self.symbols.get_indexer(s.index.get_level_values(1))
            out[d, a] = s.to_numpy(dtype=np.float64, na_value=np.nan)
        return out

    def date_mask(self, s):
        m = np.zeros(self.D, dtype=bool)
        if s is not None and len(s):
            m[self.dates.get_indexer(s.index.get_level_values(0).unique())] = True
        return m

    def symbol_mask(self, s):
        m = np.zeros(self.A, dtype=bool)
        if s is not None and len(s):
            m[self.symbols.get_indexer(pd.Index(np.asarray(s.index.get_level_values(1).unique(), dtype=object)))] = True
        return m


class Simulation:
    """Runs a daily long/short simulation given a factor series and SimulationSettings
    (portfolio_simulation.py:36-95)."""

    def __init__(self, name: str, custom_feature: pd.Series, settings: SimulationSettings):
        self.name = name
        self.custom_feature = custom_feature
        self.settings = settings
        s = settings
        self.returns = s.returns
        self.cap_flag = s.cap_flag
        self.investability_flag = s.investability_flag
        self.factors_df = s.factors_df
        self.method = s.method
        self.transaction_cost = s.transaction_cost
        self.max_weight = s.max_weight
        self.pct = s.pct
        self.min_universe = s.min_universe
        self.contributor = s.contributor
        self.output_summary = s.output_summary
        self.output_returns = s.output_returns
        self.plot = s.plot
        self.lookback_period = s.lookback_period
        self.use_cvxpy = s.use_cvxpy
        self.mvo_solver = s.mvo_solver
        self.shrinkage_intensity = s.shrinkage_intensity
        self.turnover_penalty = s.turnover_penalty
        self.return_weight = s.return_weight

    def run(self):
        """portfolio_simulation.py:73-95."""
        from portfolio_analyzer import PortfolioAnalyzer   # the reference's host reporting module
        self.factors_df[self.name] = self.custom_feature
        self.custom_feature = self.custom_feature * self.investability_flag
        weights, counts = self._daily_trade_list()
        result, top_longs, top_shorts = self._daily_portfolio_returns(weights)
        analyzer = PortfolioAnalyzer(result)
        if self.output_summary:
            metrics = self._calculate_metrics(weights, counts)
            summary_df = (pd.DataFrame.from_dict(analyzer.summary(), orient='index', columns=['Value'])
                          .reset_index().rename(columns={'index': 'Metric'}))
            print(metrics.to_string(index=False))
            print(summary_df.to_string(index=False))
        if self.contributor:
            print('Top 10 long leg contributors:', top_longs)
            print('Top 10 short leg contributors:', top_shorts)
        if self.plot:
            analyzer.plot_full_performance(counts_df=counts)
        if self.output_returns:
            return result
        return None

    # ----------------------------------------------------------------------------- trade list
    def _daily_trade_list(self):
        """portfolio_simulation.py:96-154 (equal / linear on the device)."""
        if self.method in ("mvo", "mvo_turnover"):
            return self._host_trade_list()
        if self.method not in ("equal", "linear"):
            raise ValueError(f"Unknown method {self.method}")
        return daily_trade_list(self.custom_feature, self.pct, self.method, self.max_weight)

    def _host_trade_list(self):
        """'mvo' / 'mvo_turnover': the reference's own per-date QP loop
        (portfolio_simulation.py:96-154 with :183-248, :315-746), run on a reference
        ``Simulation`` that carries this instance's state (the investability-masked signal,
        settings and any attribute changed since construction)."""
        cls, settings_cls = reference_simulation_classes()
        from dataclasses import fields
        ref_settings = settings_cls(**{f.name: getattr(self.settings, f.name) for f in fields(settings_cls)})
        ref = cls(self.name, self.custom_feature, ref_settings)
        ref.__dict__.update(self.__dict__)
        ref.settings = ref_settings
        return ref._daily_trade_list()

    @staticmethod
    def _normalize_legs(weights: pd.Series) -> pd.Series:
        """portfolio_simulation.py:250-262 (host helper, kept for API compatibility)."""
        w_pos = weights.clip(lower=0)
        w_neg = weights.clip(upper=0)
        if w_pos.sum() > 0:
            w_pos /= w_pos.sum()
        if w_neg.sum() < 0:
            w_neg /= -w_neg.sum()
        return w_pos + w_neg

    # ----------------------------------------------------------------------------- P&L
    def _daily_portfolio_returns(self, weights: pd.Series):
        """portfolio_simulation.py:748-797: per-date sums on the device over the union grid
        of the weights', returns' and cap flags' (date, symbol) cells; the reference's
        outer-join index bookkeeping on the D-length results on the host."""
        g = _Grid(weights, self.returns, self.cap_flag)
        wmask, rmask, cmask = g.date_mask(weights), g.date_mask(self.returns), g.date_mask(self.cap_flag)
        wrows = np.flatnonzero(wmask)
        wprev = np.full(g.D, -1, dtype=np.int32)
        wprev[wrows[1:]] = wrows[:-1]                      # diff() over the weights' own dates
        dev = device()
        W = torch.as_tensor(g.dense(weights), device=dev)
        R = torch.as_tensor(g.dense(self.returns), device=dev)
        CAP = torch.as_tensor(g.dense(self.cap_flag), device=dev) if self.cap_flag is not None else None
        out, contrib = E.pnl_daily(W, R, CAP, wprev, contrib=self.contributor)
        o = out.cpu().numpy()
        name = "date"
        idx_wr = pd.Index(g.dates[wmask | rmask], name=name)
        idx_wc = pd.Index(g.dates[wmask | cmask], name=name)
        idx_w = pd.Index(g.dates[wmask], name=name)
        long_ret_raw = pd.Series(o[wmask | rmask, 0], index=idx_wr)
        short_ret_raw = pd.Series(-o[wmask | rmask, 1], index=idx_wr)
        lt = pd.Series(o[wmask, 2], index=idx_w)
        st = pd.Series(o[wmask, 3], index=idx_w)
        if self.transaction_cost:
            l_cost = pd.Series(o[wmask | cmask, 4], index=idx_wc)
            s_cost = pd.Series(o[wmask | cmask, 5], index=idx_wc)
            long_ret = long_ret_raw - l_cost
            short_ret = short_ret_raw - s_cost
        else:
            long_ret, short_ret = long_ret_raw, short_ret_raw
        net = long_ret + short_ret
        result = pd.concat([
            net.rename("log_return"),
            long_ret.rename("long_return"),
            short_ret.rename("short_return"),
            lt.rename("long_turnover"),
            st.rename("short_turnover"),
            (lt + st).rename("turnover")
        ], axis=1).reset_index().sort_values("date", ascending=False).reset_index(drop=True)
        if self.contributor:
            cb = contrib.cpu().numpy()
            # the reference subtracts two Series indexed by weights ∪ returns and weights ∪
            # cap_flag symbols (:793-794): a symbol outside either set aligns to NaN, which
            # nlargest drops
            ws, rs, cs = (g.symbol_mask(s) for s in (weights, self.returns, self.cap_flag))
            cb = np.where(((ws | rs) & (ws | cs))[:, None], cb, np.nan)
            longs_pnl = pd.Series(cb[:, 0], index=g.symbols)
            shorts_pnl = pd.Series(cb[:, 1], index=g.symbols)
            return result, longs_pnl.nlargest(10), shorts_pnl.nlargest(10)
        return result, None, None

    def _calculate_metrics(self, weights: pd.Series, counts: pd.DataFrame) -> pd.DataFrame:
        """portfolio_simulation.py:799-819: daily IC of the signal against same-date returns
        (device), turnover from the weights' day-over-day changes (device)."""
        g = _Grid(self.custom_feature, self.returns)
        dev = device()
        X = torch.as_tensor(g.dense(self.custom_feature), device=dev)
        R = torch.as_tensor(g.dense(self.returns), device=dev)
        nc = E.daily_corr(X, R).cpu().numpy()
        daily_ic = pd.Series(nc[nc[:, 0] >= 1, 1])
        ic_mean, ic_std = daily_ic.mean(), daily_ic.std()
        ir = ic_mean / ic_std if ic_std else np.nan
        gw = _Grid(weights)
        wmask = gw.date_mask(weights)
        rows = np.flatnonzero(wmask)
        wprev = np.full(gw.D, -1, dtype=np.int32)
        wprev[rows[1:]] = rows[:-1]
        Wd = torch.as_tensor(gw.dense(weights), device=dev)
        o, _ = E.pnl_daily(Wd, torch.zeros_like(Wd), None, wprev)
        o = o.cpu().numpy()
        turnover_series = pd.Series(o[wmask, 2] + o[wmask, 3])
        metrics = pd.DataFrame({
            "IC (%)": [ic_mean * 100],
            "IC_IR (%)": [ir * 100],
            "IC_Std (%)": [ic_std * 100],
            "Avg Turnover (%)": [turnover_series.mean() * 100]
        })
        return round(metrics, 2)
