"""AddressSanitizer + UBSan run of the host CSV loader (SURVEY.md §5 "Race detection /
sanitizers").  ``make asan`` links csrc/csv_io.cpp with the driver
tests/asan/csv_asan_main.cpp under -fsanitize=address,undefined; the driver calls every
include/fmx_io.h entry point (mmap, multithreaded chunk parsing, sort, scatter into the
dense panel, the writer) over the CSV shapes the parity tests use (tests/test_csv_io.py),
including ragged, shuffled, CRLF and malformed files, and parses + formats every field of
a strings file.  Host-only (no GPU); the GPU kernels have no sanitizer on this pool."""
import os
import shutil
import subprocess

import numpy as np
import pandas as pd
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "factormodeling_amd", "csrc")
BIN = os.path.join(CSRC, "build_asan", "csv_asan")


@pytest.fixture(scope="module")
def driver():
    if shutil.which("g++") is None:
        pytest.skip("no host compiler")
    subprocess.run(["make", "-C", CSRC, "asan"], check=True, capture_output=True)
    return BIN


def _long(D, A, F, seed, drop=0.0, shuffle=False):
    rng = np.random.default_rng(seed)
    dates = pd.bdate_range("2015-01-01", periods=D)
    idx = pd.MultiIndex.from_product([dates, [f"S{k:05d}" for k in range(A)]], names=["date", "symbol"])
    X = rng.standard_normal((len(idx), F)) * np.exp(rng.uniform(-30, 30, (len(idx), F)))
    X[rng.random(X.shape) < 0.05] = np.nan
    df = pd.DataFrame(X, index=idx, columns=[f"f{k}" for k in range(F)])
    df["count"] = rng.integers(-50, 50, len(idx))
    if drop:
        df = df[rng.random(len(df)) >= drop]
    if shuffle:
        df = df.iloc[rng.permutation(len(df))]
    return df


def test_csv_loader_under_asan(driver, tmp_path):
    files = []
    for k, (D, A, F, drop, shuffle) in enumerate([(40, 23, 4, 0.0, False), (60, 301, 7, 0.1, True),
                                                  (3, 1, 2, 0.0, False), (120, 97, 3, 0.3, False)]):
        p = tmp_path / f"long{k}.csv"
        _long(D, A, F, k, drop, shuffle).to_csv(p)
        files += [str(p), "date", "symbol"]
    wide = tmp_path / "wide.csv"
    pd.DataFrame(np.random.default_rng(9).standard_normal((50, 6)),
                 index=pd.Index(pd.bdate_range("2020-01-01", periods=50), name="date")).to_csv(wide)
    files += [str(wide), "date", "-"]
    crlf = tmp_path / "crlf.csv"
    crlf.write_bytes(b"date,symbol,a,b\r\n2020-01-01,X,1.5,NA\r\n2020-01-01,Y,,-inf\r\n2020-01-02,X,nan,3\r\n")
    files += [str(crlf), "date", "symbol"]
    dup = tmp_path / "dup.csv"
    dup.write_text("date,symbol,a\n2020-01-01,X,1\n2020-01-01,X,2\n")
    files += [str(dup), "date", "symbol"]
    for j, text in enumerate(["date,symbol,a\n2020-01-01,X\n", "date,symbol,a\n2020-13-01,X,1\n",
                              "date,symbol,a\n2020-01-01,X,abc\n", "", "date,symbol,a\n",
                              "date,symbol,a\n2020-01-01,\"X\",1\n", "date,symbol,a\n2020-01-01,X,1e400e\n"]):
        bad = tmp_path / f"bad{j}.csv"
        bad.write_text(text)
        files += [str(bad), "date", "symbol"]
    rng = np.random.default_rng(4)
    v = rng.standard_normal(20000) * np.exp(rng.uniform(-300, 300, 20000))
    fields = [repr(float(x)) for x in v] + ["%.25e" % x for x in v[:2000]] + ["%.40f" % x for x in v[:500]]
    fields += ["", " ", "-", "+", ".", "e5", "1e", "1e+", "nan", "-inf", "Infinity", "1" * 400, "0." + "0" * 350 + "1",
               "9" * 30 + "e-330", "4.9e-324", "1e-400", "  7  ", "\t1.5"]
    sf = tmp_path / "fields.txt"
    sf.write_text("\n".join(fields) + "\n")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([driver, str(sf), "4"] + files, capture_output=True, text=True, env=env, timeout=300)
    log = r.stdout + r.stderr
    assert "AddressSanitizer" not in log and "runtime error" not in log, log[-4000:]
    assert r.returncode == 0, log[-4000:]
    assert "asan driver ok" in r.stdout
    assert f"fields {len(fields)}" in r.stdout
