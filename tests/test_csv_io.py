"""Native long-CSV loader (csrc/csv_io.cpp) vs the reference's pandas loading step.

Oracle: pandas 2.3.3 in this container, called exactly as pipeline.ipynb:71-82 does
(pd.read_csv, pd.to_datetime(date), set_index([date, symbol])).  pandas' default float
parser (tokenizer.c precise_xstrtod) is not correctly rounded, so these tests also pin the
restatement bit-for-bit on values where it differs from strtod.  Host-only: no GPU.
"""
import io
import os

import numpy as np
import pandas as pd
import pytest

from factormodeling_amd import csv_io
from factormodeling_amd.panel import PanelIndex


def _ref_load(path, symbol=True):
    df = pd.read_csv(path)
    df["date"] = pd.to_datetime(df["date"])
    df.set_index(["date", "symbol"] if symbol else ["date"], inplace=True)
    return df


def _long_frame(D=30, A=17, F=5, seed=0, drop=0.0, shuffle=False):
    rng = np.random.default_rng(seed)
    dates = pd.bdate_range("2015-01-01", periods=D)
    syms = [f"S{k:05d}" for k in rng.permutation(A)]
    idx = pd.MultiIndex.from_product([dates, sorted(syms)], names=["date", "symbol"])
    X = rng.standard_normal((len(idx), F))
    X[rng.random(X.shape) < 0.05] = np.nan
    X[:, 1] *= 1e-7
    X[:, 2] = np.round(X[:, 2], 2)
    cols = [f"g{f // 4:03d}_{f:04d}_{'eq flx long short raw'.split()[f % 5]}" for f in range(F)]
    df = pd.DataFrame(X, index=idx, columns=cols)
    df["count"] = rng.integers(-50, 50, len(idx))
    if drop:
        df = df[rng.random(len(df)) >= drop]
    if shuffle:
        df = df.iloc[rng.permutation(len(df))]
    return df


def test_library_exports_every_declared_symbol():
    import re
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "fmx_io.h")).read()
    declared = set(re.findall(r"\b(fmx_\w+)\s*\(", hdr))
    lib = csv_io.load()
    for name in declared:
        assert hasattr(lib, name), name
    assert declared == set(csv_io.SIGNATURES)


def test_float_parser_matches_pandas_default_bitwise():
    rng = np.random.default_rng(3)
    v = rng.standard_normal(60000) * np.exp(rng.uniform(-40, 40, 60000))
    strs = [repr(float(x)) for x in v] + ["%.6g" % x for x in v[:5000]] + ["%.20e" % x for x in v[:5000]]
    strs += ["%.25f" % x for x in v[:3000]] + ["1e-320", "4.9e-324", "2.5e-310", "1.7976931348623157e308",
                                               "-0", "+5", " 3.5 ", "1E+5", "12345678901234567.5", "1.e3",
                                               ".5", "5.", "0.000000000000000000000123456789012345678",
                                               "9223372036854775807", "1e-400"]
    ref = pd.read_csv(io.StringIO("x\n" + "\n".join(strs) + "\n"))["x"].to_numpy()
    assert ref.dtype == np.float64
    got = np.array([csv_io.parse_double(s) for s in strs], dtype=np.float64)
    rt = np.array([float(s) for s in strs])
    assert (ref != rt).sum() > 1000  # the default parser is not correctly rounded ...
    np.testing.assert_array_equal(got.view(np.int64), ref.view(np.int64))  # ... and we match it


@pytest.mark.parametrize("field", ["1e", "1e+", "1e400", "-", ".", "abc"])
def test_unparseable_fields_raise(tmp_path, field):
    p = tmp_path / "bad.csv"
    p.write_text(f"date,symbol,x\n2015-01-01,A,1.5\n2015-01-02,A,{field}\n")
    assert pd.read_csv(p)["x"].dtype == object  # pandas gives up on the column too
    with pytest.raises(csv_io.FmxIOError, match="data row 1"):
        csv_io.read_long_csv(p)


@pytest.mark.parametrize("drop,shuffle", [(0.0, False), (0.1, False), (0.1, True)])
def test_read_long_csv_equals_reference_loading(tmp_path, drop, shuffle):
    df = _long_frame(drop=drop, shuffle=shuffle)
    p = tmp_path / "factors.csv"
    df.to_csv(p)
    ref = _ref_load(p)
    for threads in (1, 3, 8):
        got = csv_io.read_long_csv(p, threads=threads)
        pd.testing.assert_frame_equal(got, ref, check_exact=True)
        assert got["count"].dtype == np.int64


def test_na_spellings_and_crlf(tmp_path):
    nas = ["", "NaN", "nan", "NA", "N/A", "NULL", "null", "None", "<NA>", "#N/A", "-nan", "1.#QNAN"]
    lines = ["date,symbol,x,y"] + [f"2015-01-{d + 1:02d},S{k},{nas[(d * 3 + k) % len(nas)]},{d}.{k}"
                                   for d in range(12) for k in range(3)]
    lines += ["2015-01-20,S0,inf,-Infinity", "2015-01-20,S1,1e5,+7", "2015-01-20,S2, 2.5 ,-0"]
    p = tmp_path / "na.csv"
    p.write_bytes(("\r\n".join(lines) + "\r\n").encode())
    pd.testing.assert_frame_equal(csv_io.read_long_csv(p), _ref_load(p), check_exact=True)


def test_datetime_dates_and_wide_file(tmp_path):
    rng = np.random.default_rng(5)
    dates = pd.date_range("2020-03-01 09:30:00", periods=40, freq="37min")
    df = pd.DataFrame(0.01 * rng.standard_normal((40, 6)), index=pd.Index(dates, name="date"),
                      columns=[f"f{k}" for k in range(6)])
    p = tmp_path / "single_factor_returns.csv"
    df.to_csv(p)
    ref = _ref_load(p, symbol=False)
    got = csv_io.read_long_csv(p, symbol_col=None)
    pd.testing.assert_frame_equal(got, ref, check_exact=True)
    pan = csv_io.load_panel(p, symbol_col=None)
    np.testing.assert_array_equal(pan.X[:, :, 0], ref.to_numpy().T)  # text round trip: pandas values


@pytest.mark.parametrize("drop", [0.0, 0.15])
def test_load_panel_equals_panel_index_dense(tmp_path, drop):
    df = _long_frame(D=25, A=40, F=7, seed=2, drop=drop)
    p = tmp_path / "f.csv"
    df.to_csv(p)
    ref = _ref_load(p)
    pi = PanelIndex(ref.index)
    want = pi.to_dense(ref.to_numpy(dtype=np.float64))
    pan = csv_io.load_panel(p, threads=4)
    assert pan.per_symbol_sorted
    assert list(pan.names) == list(ref.columns)
    pd.testing.assert_index_equal(pan.dates, pi.dates.rename("date"))
    assert list(pan.symbols) == list(pi.symbols)
    np.testing.assert_array_equal(pan.X, want)


def test_integer_symbols_sorted_numerically(tmp_path):
    p = tmp_path / "ints.csv"
    p.write_text("date,symbol,x\n2015-01-01,10,1.0\n2015-01-01,9,2.0\n2015-01-02,10,3.0\n2015-01-02,9,4.0\n")
    ref = _ref_load(p)
    pd.testing.assert_frame_equal(csv_io.read_long_csv(p), ref, check_exact=True)
    pan = csv_io.load_panel(p)
    assert list(pan.symbols) == [9, 10]
    np.testing.assert_array_equal(pan.X[0], [[2.0, 1.0], [4.0, 3.0]])


def test_duplicates_and_unsorted_rows_flagged(tmp_path):
    p = tmp_path / "dup.csv"
    p.write_text("date,symbol,x\n2015-01-02,A,1.0\n2015-01-01,A,2.0\n2015-01-02,A,3.0\n")
    with pytest.raises(csv_io.FmxIOError, match="duplicate"):
        csv_io.load_panel(p)
    p.write_text("date,symbol,x\n2015-01-02,A,1.0\n2015-01-01,A,2.0\n")
    assert not csv_io.load_panel(p).per_symbol_sorted


@pytest.mark.parametrize("text,msg", [
    ("date,symbol,x\n2015-01-01,A,1,2\n", "more fields"),
    ("date,symbol,x\n2015-01-01,A\n", "fields"),
    ('date,symbol,x\n2015-01-01,"A",1\n', "quoted"),
    ("date,symbol,x\n01/02/2015,A,1\n", "ISO"),
    ("sym,x\nA,1\n", "lacks column"),
    ("date,symbol,x\n2015-01-01,NA,1\n", "NA spellings"),     # pandas: NaN symbol
    ("date,symbol,x\n2015-01-01,,1\n", "NA spellings"),
    ("date,symbol,x\n2015-01-01,null,1\n", "NA spellings"),
    ("date,symbol,x,x\n2015-01-01,A,1,2\n", "duplicate header"),  # pandas: 'x', 'x.1'
    ("date,symbol,x\nNA,A,1\n", "ISO"),
])
def test_format_errors_are_loud(tmp_path, text, msg):
    p = tmp_path / "e.csv"
    p.write_text(text)
    with pytest.raises(csv_io.FmxIOError, match=msg):
        csv_io.read_long_csv(p)


def test_missing_file_raises(tmp_path):
    with pytest.raises(csv_io.FmxIOError, match="cannot open"):
        csv_io.read_long_csv(tmp_path / "absent.csv")


def test_format_double_is_python_repr():
    rng = np.random.default_rng(9)
    vals = list(rng.standard_normal(20000) * np.exp(rng.uniform(-60, 60, 20000)))
    vals += [0.0, -0.0, 1.0, 123.0, 1e16, 1e15, 9999999999999998.0, 1e-4, 1e-5, 0.00012, 1e22, 5e-324,
             1.7976931348623157e308, np.inf, -np.inf, 0.1, 1 / 3, 2.5e-310, -1234.5]
    for v in vals:
        assert csv_io.format_double(v) == repr(float(v)), v
    assert csv_io.format_double(np.nan) == ""


@pytest.mark.parametrize("drop", [0.0, 0.2])
def test_write_long_csv_bytes_equal_to_csv(tmp_path, drop):
    df = _long_frame(D=20, A=15, F=6, seed=4, drop=drop).drop(columns=["count"])
    df.iloc[3, 2] = np.inf
    df.iloc[4, 1] = 1e16
    a, b = tmp_path / "ref.csv", tmp_path / "got.csv"
    df.to_csv(a)
    csv_io.write_long_csv(df, b, threads=3)
    assert b.read_bytes() == a.read_bytes()
    # composite factor Series and date-indexed weights (pipeline.ipynb:391,464)
    s = df.iloc[:, 0].rename("composite_factor")
    s.to_csv(a)
    csv_io.write_long_csv(s, b)
    assert b.read_bytes() == a.read_bytes()
    w = pd.DataFrame(np.random.default_rng(1).random((12, 4)), columns=pd.Index(list("abcd"), name="factor"),
                     index=pd.Index(pd.bdate_range("2016-01-01", periods=12), name="date"))
    w.iloc[2] = 0.0
    w.to_csv(a)
    csv_io.write_long_csv(w, b)
    assert b.read_bytes() == a.read_bytes()
    # and it reads back through the native loader to the same frame pandas reads
    pd.testing.assert_frame_equal(csv_io.read_long_csv(b, symbol_col=None), _ref_load(a, symbol=False),
                                  check_exact=True)


def test_write_long_csv_rejects_unsupported(tmp_path):
    df = _long_frame(D=5, A=4, F=3)
    with pytest.raises(ValueError, match="float64"):
        csv_io.write_long_csv(df, tmp_path / "x.csv")  # int column
    with pytest.raises(ValueError, match="order"):
        csv_io.write_long_csv(df.drop(columns=["count"]).iloc[::-1], tmp_path / "x.csv")


@pytest.mark.gpu
def test_load_panel_to_hbm_feeds_the_engine(tmp_path):
    """CSV -> pinned host -> HBM -> cs_rank / ts_mean kernels, checked against the oracle
    on the pandas-loaded panel."""
    import torch

    import factormodeling_amd.engine as E
    import oracle.ops as O
    df = _long_frame(D=40, A=300, F=3, seed=6, drop=0.0).drop(columns=["count"])
    p = tmp_path / "f.csv"
    df.to_csv(p)
    ref = _ref_load(p)
    want = PanelIndex(ref.index).to_dense(ref.to_numpy(dtype=np.float64))
    pan = csv_io.load_panel(p, device="cuda:0")
    assert isinstance(pan.X, torch.Tensor) and pan.X.is_cuda
    np.testing.assert_array_equal(pan.X.cpu().numpy(), want)
    rk = E.cs_rank(pan.X).cpu().numpy()
    mu = E.ts("mean", pan.X, 5).cpu().numpy()
    for f in range(want.shape[0]):
        np.testing.assert_array_equal(rk[f], O.cs_rank(want[f]))
        np.testing.assert_array_equal(mu[f], O.ts_mean(want[f], 5))
