"""The fp32 division identity the apply kernels use (smaq_elem.h div_by_const):
RN32(RN64(a * RN64(1/b))) == RN32(a / b) whenever the quotient is 0 or a normal fp32 number.
Checked on the host CPU (IEEE binary64/binary32 like the GPU's v_mul_f64 / v_cvt_f32_f64) with
oracle/csrc/div_check.c: random operand pairs across all exponents, and every one of the 2^32
fp32 dividends against a SmaQ range constant."""

import json
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_div_identity(tmp_path):
    exe = str(tmp_path / "div_check")
    subprocess.check_call(["gcc", "-O2", "-fopenmp", "-ffp-contract=off",
                           os.path.join(REPO, "oracle", "csrc", "div_check.c"), "-o", exe, "-lm"])
    r = json.loads(subprocess.check_output([exe, "random", "50000000"]))
    assert r["mismatches"] == 0 and r["checked"] > 4.9e7
    r = json.loads(subprocess.check_output([exe, "all", "15"]))
    assert r["mismatches"] == 0 and r["checked"] > 4.2e9


def test_div_identity_subnormal_quotients(tmp_path):
    """Subnormal quotients (smaq_elem.h quot_check_for): exact for every divisor that is neither an
    even integer nor >= 2^24, so those calls skip the per-element check; the checked divisors are
    exercised too (they keep the IEEE fallback on the GPU)."""
    exe = str(tmp_path / "div_check")
    subprocess.check_call(["gcc", "-O2", "-fopenmp", "-ffp-contract=off",
                           os.path.join(REPO, "oracle", "csrc", "div_check.c"), "-o", exe, "-lm"])
    r = json.loads(subprocess.check_output([exe, "subrand", "1000000"]))
    assert r["mismatches"] == 0 and r["checked"] > 2.5e7
    r = json.loads(subprocess.check_output([exe, "sub", "3", "0.7", "1.3e-5"]))
    assert r["mismatches"] == 0 and r["checked"] > 5e7
