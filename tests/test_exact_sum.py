"""The exact fixed-point accumulator behind the GPU-count-independent Gram
(csrc/exactsum.hpp, fmx_gram_exact): the library's host run of the device code against
the numpy restatement (oracle/gram.py), bit for bit; order/grouping independence; and
accuracy against math.fsum."""
import ctypes
import math
import os

import numpy as np
import pytest

import oracle.gram as OG


def _lib():
    from factormodeling_amd import _lib as L
    if not os.path.exists(L.LIB_PATH):
        pytest.skip("libfmx.so not built")
    return L.load()


def _cfold(x):
    lib = _lib()
    x = np.ascontiguousarray(x, dtype=np.float64)
    limbs = np.zeros(OG.EX_SLOTS, dtype=np.int64)
    v = ctypes.c_double()
    lib.fmx_debug_exact_fold(x.ctypes.data_as(ctypes.c_void_p), x.size, limbs.ctypes.data_as(ctypes.c_void_p),
                             ctypes.byref(v))
    return limbs, v.value


def _values(rng, n):
    x = rng.standard_normal(n) * np.exp(rng.uniform(-30, 30, n))
    x[::7] = np.round(x[::7], 2)
    x[::11] *= -1
    x[5::13] = 0.0
    x[3::17] = -0.0
    x[1::19] = 5e-324 * rng.integers(1, 100, x[1::19].size)   # subnormals (dropped below 2^-64)
    return x


@pytest.mark.parametrize("seed", range(6))
def test_host_device_code_matches_numpy_restatement(seed):
    rng = np.random.default_rng(seed)
    x = _values(rng, 3000)
    limbs_c, v_c = _cfold(x)
    limbs_np = OG.ex_fold(x[:, None])[:, 0]
    # both un-normalised accumulations of the same chunks: identical integer limbs
    assert np.array_equal(limbs_c, limbs_np)
    v_np = OG.ex_value(limbs_np[:, None])[0]
    assert v_c == v_np or (math.isnan(v_c) and math.isnan(v_np))


def test_order_and_grouping_independent():
    rng = np.random.default_rng(7)
    x = _values(rng, 4096) * 1e3
    ref = OG.ex_value(OG.ex_fold(x[:, None]))[0]
    for k in range(5):
        p = rng.permutation(x)
        cuts = np.sort(rng.choice(np.arange(1, x.size), size=k + 1, replace=False))
        groups = np.split(p, cuts)
        tot = sum(OG.ex_fold(g[:, None]) for g in groups)          # per-rank limbs, then integer sum
        assert OG.ex_value(tot)[0] == ref
        assert _cfold(p)[1] == ref


def test_accuracy_vs_fsum():
    rng = np.random.default_rng(3)
    for scale in (1.0, 1e4, 1e-6):
        x = rng.standard_normal(20000) * scale
        got = OG.ex_value(OG.ex_fold(x[:, None]))[0]
        ref = math.fsum(x)
        # truncation at 2^-64 per term + one Horner rounding per limb
        assert abs(got - ref) <= 20000 * 2.0 ** -64 + 4 * abs(ref) * 2.0 ** -52


def test_flags_nonfinite_and_out_of_range():
    assert math.isnan(_cfold(np.array([1.0, np.inf]))[1])
    assert math.isnan(_cfold(np.array([1.0, np.nan]))[1])
    assert math.isnan(_cfold(np.array([2.0 ** 130]))[1])
    assert _cfold(np.array([2.0 ** 120, -2.0 ** 120, 3.0]))[1] == 3.0
    assert math.isnan(OG.ex_value(OG.ex_fold(np.array([[np.inf]])))[0])


def test_gram_exact_parts_split_invariant():
    """The oracle's exact Gram: any split of the dates into shards sums to the same limbs."""
    rng = np.random.default_rng(1)
    X = rng.standard_normal((5, 40, 30))
    X[rng.random(X.shape) < 0.05] = np.nan
    Z, M = OG.zscore_exposures(X)
    L1, N1 = OG.gram_exact_parts(Z, M)
    for cuts in ([20], [7, 19, 33], [1, 2, 3, 39]):
        bounds = [0] + cuts + [40]
        parts = [OG.gram_exact_parts(Z, M, a, b) for a, b in zip(bounds[:-1], bounds[1:])]
        L = sum(p[0] for p in parts)
        N = sum(p[1] for p in parts)
        assert np.array_equal(OG.ex_value(L), OG.ex_value(L1)) and np.array_equal(N, N1)
    G, Nf = OG.gram_exact_finalize(L1, N1)
    Zf, Mf = Z.reshape(5, -1), M.reshape(5, -1)
    np.testing.assert_allclose(G, Zf @ Zf.T, rtol=1e-13, atol=1e-12)
    assert np.array_equal(Nf, Mf @ Mf.T)
