"""The numpy oracle behind factormodeling_amd.pipeline's backend interface (test
infrastructure only: the gloo sharding test and the GPU step-level parity test compare
the product's EngineBackend against it)."""
import numpy as np
import torch

import oracle.gram as OG
import oracle.metrics as OM
import oracle.ops as O


class OracleBackend:
    """numpy oracle behind the pipeline's backend interface (tests only)."""

    def op(self, kind, op, w, X, out):
        x = X.numpy()
        for f in range(x.shape[0]):
            if kind == "ts":
                fn = {"mean": O.ts_mean, "std": O.ts_std, "zscore": O.ts_zscore, "rank": O.ts_rank,
                      "decay": O.ts_decay}[op]
                r = fn(x[f], w)
            elif kind == "cs_rank":
                r = O.cs_rank(x[f])
            elif kind == "cs":
                r = {"zscore": O.cs_zscore, "market_neutralize": O.market_neutralize}[op](x[f])
            else:
                r = O.cs_winsor(x[f])
            out[f] = torch.from_numpy(r)
        return out

    def ts_corr_into(self, X, R, w, out):
        x, r = X.numpy(), R.numpy()
        for f in range(x.shape[0]):
            out[f] = torch.from_numpy(O.ts_corr(x[f], r, w))
        return out

    def corr_vol_feature(self, X, C, w, out):
        """sign(C) * x / ts_std(x, w) with C = the step's ts_corr (oracle.ops.corr_vol_feature)."""
        x, c = X.numpy(), C.numpy()
        for f in range(x.shape[0]):
            s = O.ts_std(x[f], w)
            with np.errstate(all="ignore"):
                out[f] = torch.from_numpy(np.sign(c[f]) * (x[f] / np.where(s == 0, np.nan, s)))
        return out

    def corr_feature_into(self, X, R, w, out, corr_out=None):
        """The fused pass: ts_corr then the feature (the oracle has no fusion to mirror)."""
        c = self.ts_corr_into(X, R, w, torch.empty_like(X) if corr_out is None else corr_out)
        return self.corr_vol_feature(X, c, w, out)

    def weighted_composite(self, X, names, pdate, w, method):
        """weighted_composite_factor of each processed day's selection (owned dates only)."""
        import oracle.composite as OC
        own = np.asarray(pdate) >= 0
        W = w.numpy() if isinstance(w, torch.Tensor) else np.asarray(w)
        out = OC.weighted_composite_factor(X.numpy(), names, list(np.asarray(pdate)[own]), W[own], method)
        return torch.from_numpy(out)

    def ic_daily(self, X, R, lags):
        x, r = X.numpy(), R.numpy()
        Fn, Dn, _ = x.shape
        out = np.full((len(lags), 4, Fn, Dn), np.nan)
        out[:, 0] = 0
        for li, L in enumerate(lags):
            for f in range(Fn):
                for t in range(L, Dn):
                    out[li, :, f, t] = OM.daily_stats(x[f, t - L], r[t])
        return torch.from_numpy(out)

    def ic_window(self, daily, d0s, d1s):
        dl = daily.numpy()
        Fn = dl.shape[1]
        out = np.full((len(d0s), Fn, 8), np.nan)
        for j, (a, b) in enumerate(zip(d0s, d1s)):
            for f in range(Fn):
                sel = dl[0, f, a:b] >= 3
                ic, ric, be = dl[1, f, a:b][sel], dl[2, f, a:b][sel], dl[3, f, a:b][sel]
                out[j, f, :7] = OM.summarize(ic, ric, be)
                out[j, f, 5] = np.sum(~np.isnan(be))
        return torch.from_numpy(out)

    def select_icir_top(self, metrics, use_rank, thr, top_x):
        m = metrics.numpy()
        J, Fn, _ = m.shape
        w = np.zeros((J, Fn))
        order = np.zeros((J, Fn), np.int32)
        for j in range(J):
            o = OM.nargsort_desc(m[j, :, 3])
            order[j] = o
            w[j, o] = OM.icir_top(o, m[j], thr, top_x, use_rank)
        return torch.from_numpy(order), torch.from_numpy(w)

    def zscore_exposures(self, X):
        Z, M = OG.zscore_exposures(X.numpy())
        return torch.from_numpy(Z), torch.from_numpy(M)

    def corr_gram_exact(self, X, d0, d1, stats=None, z=None):
        """Exact fixed-point Gram partials of dates [d0, d1) (one fold unit per date)."""
        Z, M = OG.zscore_exposures(X[:, d0:d1].numpy())
        limbs, counts = OG.gram_exact_parts(Z, M)
        return torch.from_numpy(limbs), torch.from_numpy(counts)

    @staticmethod
    def gram_exact_finalize(limbs, counts):
        G, N = OG.gram_exact_finalize(limbs.numpy(), counts.numpy())
        return torch.from_numpy(G), torch.from_numpy(N)

    def gram(self, Z, M):
        Zf = Z.reshape(Z.shape[0], -1).double()
        Mf = M.reshape(M.shape[0], -1).double()
        return Zf @ Zf.T, Mf @ Mf.T

    @staticmethod
    def greedy_prune(C, order, rho, top_x):
        Cn = C.numpy() if isinstance(C, torch.Tensor) else C
        return OG.greedy_prune(Cn, order, rho, top_x)
