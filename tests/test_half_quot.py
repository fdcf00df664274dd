"""The two-op fp32 quotient q / range of the half-input apply (smaq_elem.h quot_split_compute,
include/smq.h smq_half_quot_split) against its restatement in oracle/csrc/half_div_check.c (qr
mode), which enumerates every code the flags can produce from a half z-score (smart.py:154-171)
and compares fmaf(q, h, q * l) with the fp64-derived IEEE quotient. CPU only: the library's host
check decides which form the device launch takes."""

import ctypes
import pathlib
import random
import subprocess

import numpy as np
import pytest

from helpers import smaq_hparams

REPO = pathlib.Path(__file__).resolve().parent.parent

pytestmark = pytest.mark.timeout(300)


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = tmp_path_factory.mktemp("qr") / "half_div_check"
    src = REPO / "oracle" / "csrc" / "half_div_check.c"
    subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", str(src), "-o", str(exe), "-lm"],
                   check=True)
    return exe


def _oracle(exe, dt, thr, rm, ro, sr):
    out = subprocess.run([str(exe), "qr", dt, repr(float(thr)), float(rm).hex(), float(ro).hex(),
                          str(int(sr))], check=True, capture_output=True, text=True).stdout.split()
    return int(out[0]), [float.fromhex(v) for v in out[1:]]


def _lib(dt, thr, rm, ro, sr):
    from smart_compress_amd import _native as N

    out = (ctypes.c_float * 4)()
    code = N.SMQ_DTYPE_F16 if dt == "f16" else N.SMQ_DTYPE_BF16
    ok = N.lib().smq_half_quot_split(code, thr, rm, ro, int(sr), out)
    return ok, [float(v) for v in out]


def _ranges(hp):
    from smart_compress_amd.compress.smart import SmartFP

    c = SmartFP(hp)
    return (float(np.float32(c.range_normal)), float(np.float32(c.range_outlier)))


def test_default_flags_take_the_fp32_form(checker):
    """precision=16 with the default flags (the half bench configuration): both half types pass,
    in the library and in the oracle, with the same split constants."""
    hp = smaq_hparams(precision=16)
    rm, ro = _ranges(hp)
    thr = float(np.float32(hp.main_std_dev_threshold))
    for dt in ("f16", "bf16"):
        ok, v = _lib(dt, thr, rm, ro, True)
        ok_o, v_o = _oracle(checker, dt, thr, rm, ro, True)
        assert ok == ok_o == 1
        assert np.array_equal(np.float32(v), np.float32(v_o))


def test_library_agrees_with_oracle_on_flag_sets(checker):
    """Random SmaQ flag sets (bits 3-16, thresholds 0.25-6, both rounding modes): the library's
    verdict and split constants equal the oracle's."""
    rs = random.Random(5)
    cases = []
    for _ in range(24):
        bm = rs.randint(3, 12)
        bo = rs.randint(bm, 16)
        tm = rs.choice([0.25, 0.5, 1.0, 1.3, 1.5, 2.0, 2.7, 3.0, 4.0])
        to = tm + rs.choice([0.1, 0.5, 1.0, 2.5, 6.0])
        cases.append((rs.choice(["f16", "bf16"]), bm, bo, tm, to, rs.random() < 0.7))
    verdicts = set()
    for dt, bm, bo, tm, to, sr in cases:
        hp = smaq_hparams(precision=16, num_bits_main=bm, num_bits_outlier=bo,
                          main_std_dev_threshold=tm, outlier_std_dev_threshold=to,
                          stochastic_rounding=sr)
        rm, ro = _ranges(hp)
        thr = float(np.float32(tm))
        ok, v = _lib(dt, thr, rm, ro, sr)
        ok_o, v_o = _oracle(checker, dt, thr, rm, ro, sr)
        assert ok == ok_o, (dt, bm, bo, tm, to, sr)
        assert np.array_equal(np.float32(v), np.float32(v_o))
        verdicts.add((sr, ok))
    assert (True, 1) in verdicts


def test_stochastic_sweep_passes(checker):
    """The oracle's sweep over 17,640 flag sets: every stochastic-rounding set passes (truncating
    sets with l < 0 fail at q = +-inf and keep the fp64 form)."""
    out = subprocess.run([str(checker), "qr-sweep"], check=True, capture_output=True,
                         text=True).stdout.strip().splitlines()[-1]
    sets, sr_sets, sr_ok = (int(v) for v in np.array(out.replace(",", "").replace(";", "").split())[
        [1, 8, 10]])
    assert sets == 17640 and sr_sets == sr_ok == 8820, out
