"""The reciprocal-table division behind k_ts_corr_fast (ts_ops.hip mdiv: q0 = RN(x r),
rem = fma(-q0, n, x), q = fma(rem, r, q0) with r = RN(1/n)) returns the IEEE quotient x / n
bit for bit: 8e7 host cases (tests/native/mdiv_check.c, the same arithmetic with libm's
correctly rounded fma), including x within a few ulps of multiples of n, where q0 is off by
more than an ulp.  The GPU side is pinned by the bit-exact ts_corr tests."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def test_mdiv_matches_ieee_division(tmp_path):
    exe = tmp_path / "mdiv_check"
    try:
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), os.path.join(HERE, "native", "mdiv_check.c"),
                        "-lm"], check=True, capture_output=True)
    except (OSError, subprocess.CalledProcessError) as e:
        pytest.skip(f"no host C compiler: {e}")
    p = subprocess.run([str(exe), "4096", "20000"], capture_output=True, text=True)
    assert p.returncode == 0, p.stderr + p.stdout
    assert "0 mismatches" in p.stdout


def test_rdiv_matches_ieee_division(tmp_path):
    """fmx_common.hpp rdiv (the cross-sectional z-scores' (x - mean) / sd from RN(1 / sd):
    Markstein's correction for a general divisor, with its range guards) == the IEEE
    quotient on 1e8 host cases (tests/native/rdiv_check.c)."""
    exe = tmp_path / "rdiv_check"
    try:
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), os.path.join(HERE, "native", "rdiv_check.c"),
                        "-lm"], check=True, capture_output=True)
    except (OSError, subprocess.CalledProcessError) as e:
        pytest.skip(f"no host C compiler: {e}")
    p = subprocess.run([str(exe), "25000", "4000"], capture_output=True, text=True)
    assert p.returncode == 0, p.stderr + p.stdout
    assert "0 mismatches" in p.stdout
