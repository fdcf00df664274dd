"""S2FP8 (smart_compress/compress/s2fp8.py:27-48) restated in numpy float32."""

import numpy as np

from . import qtorch_float as qf

F32 = np.float32


def stats(x: np.ndarray):
    """s2fp8.py:31-43 -> dict(mu, m, alpha, beta, beta_pow2, inv_beta_pow2, inv_alpha)."""
    a = np.abs(np.asarray(x, dtype=F32))
    with np.errstate(all="ignore"):
        lg = np.where(a == F32(0), a, np.log2(a)).astype(F32)
    mu = F32(np.mean(lg.astype(np.float64)))
    m = F32(np.max(lg))
    return derive(mu, m)


def derive(mu, m):
    mu, m = F32(mu), F32(m)
    with np.errstate(all="ignore"):
        alpha = (F32(1) / (m - mu)) * F32(15.0)  # Tensor.__rtruediv__ = reciprocal() * 15.0
        beta = (-alpha) * mu
        bp2 = F32(np.exp2(np.float64(beta)))
        return dict(mu=mu, m=m, alpha=alpha, beta=beta, beta_pow2=bp2,
                    inv_beta_pow2=F32(1) / bp2, inv_alpha=F32(1) / alpha)


def transform(x, st):
    """Y = |x|^alpha * 2^beta (s2fp8.py:45), the quantiser's input."""
    a = np.abs(np.asarray(x, dtype=F32))
    with np.errstate(all="ignore"):
        return (np.power(a, st["alpha"]).astype(F32) * st["beta_pow2"]).astype(F32)


def inverse(T, x, st):
    """((T * 2^-beta) ** (1/alpha)) * sign(x) (s2fp8.py:46-48); torch.sign(+-0, NaN) = +0."""
    x = np.asarray(x, dtype=F32)
    sgn = np.where(x > 0, F32(1), np.where(x < 0, F32(-1), F32(0))).astype(F32)
    with np.errstate(all="ignore"):
        t1 = (np.asarray(T, dtype=F32) * st["inv_beta_pow2"]).astype(F32)
        t2 = np.power(t1, st["inv_alpha"]).astype(F32)
        return (t2 * sgn).astype(F32)


def roundtrip(x, rand_bits, check_inf_flag=True, st=None):
    st = stats(x) if st is None else st
    Y = transform(x, st)
    T = qf.float_quantize(Y, 5, 2, rand_bits, check_inf_flag)
    return inverse(T, x, st), st, Y, T


# ---- precision 16 (Lightning half training) --------------------------------------------------------
# s2fp8.py:27-48 with quantization.py:187-204's `is_16_bit` branch, op for op in the dtypes torch
# (CPU, 2.10) uses. P = the input's type ('f32' | 'f16' | 'bf16'):
#   * statistics and forward transform in P: every op is its fp32 value rounded to P (torch CPU
#     computes reduced-precision ops in fp32 and rounds once; the mean rounds its fp32 quotient);
#   * float_quantize quantises Y.float() and returns .half() (E5M2 values are exact in half);
#   * `truncated * beta_pow2.reciprocal_()`: half tensor times a 0-dim P scalar -> half, computed
#     from the UNROUNDED scalar (torch's opmath path for CPU scalars);
#   * `** alpha.reciprocal_()`: the exponent is rounded to half first, the power rounded to half;
#   * `* signs`: half * P -> half for P = f16, fp32 otherwise (type promotion of two tensors).
# Pinned by tests/golden/s2p16_*.npz (make_golden.py gen_s2fp8_p16). The CUDA reference may differ
# in the scalar corner above (a GPU 0-dim tensor is cast to half); not measurable here.

def _r(v, dt):
    from .smaq import round_to

    return round_to(v, dt)


def stats_p16(x, dt: str):
    a = np.abs(np.asarray(x, dtype=F32))
    with np.errstate(all="ignore"):
        lg = _r(np.where(a == F32(0), a, np.log2(a)).astype(F32), dt)
    mu = _r(F32(np.mean(lg.astype(np.float64))), dt)
    m = F32(np.max(lg))
    return derive_p16(mu, m, dt)


def derive_p16(mu, m, dt: str):
    mu, m = F32(mu), F32(m)
    with np.errstate(all="ignore"):
        t = _r(m - mu, dt)
        alpha = _r(_r(F32(1) / t, dt) * F32(15.0), dt)  # reciprocal() * 15.0, both in P
        beta = _r((-alpha) * mu, dt)
        bp2 = _r(F32(np.exp2(np.float64(beta))), dt)
        return dict(mu=mu, m=m, alpha=alpha, beta=beta, beta_pow2=bp2,
                    inv_beta_pow2=_r(F32(1) / bp2, dt), inv_alpha=_r(F32(1) / alpha, dt))


def transform_p16(x, st, dt: str):
    a = np.abs(np.asarray(x, dtype=F32))
    with np.errstate(all="ignore"):
        Y = _r(np.power(a.astype(np.float64), np.float64(st["alpha"])).astype(F32), dt)
        return _r(Y * st["beta_pow2"], dt)


def inverse_p16(T, x, st, dt: str):
    """-> output values (float32 array) and the output type ('f16' for f16 inputs, else 'f32')."""
    x = np.asarray(x, dtype=F32)
    sgn = np.where(x > 0, F32(1), np.where(x < 0, F32(-1), F32(0))).astype(F32)
    th = _r(np.asarray(T, dtype=F32), "f16")  # .half(): exact for E5M2 values, inf, NaN
    ia = _r(st["inv_alpha"], "f16")
    with np.errstate(all="ignore"):
        t1 = _r(th * st["inv_beta_pow2"], "f16")
        t2 = _r(np.power(t1.astype(np.float64), np.float64(ia)).astype(F32), "f16")
        return (t2 * sgn).astype(F32), ("f16" if dt == "f16" else "f32")


def roundtrip_p16(x, dt: str, rand_bits, check_inf_flag=True, st=None):
    st = stats_p16(x, dt) if st is None else st
    Y = transform_p16(x, st, dt)
    T = qf.float_quantize(Y, 5, 2, rand_bits, check_inf_flag)
    y, out_dt = inverse_p16(T, x, st, dt)
    return y, out_dt, st, Y, T


# ---- float64 data --------------------------------------------------------------------------------
# s2fp8.py:27-48 on a float64 tensor: the log2 statistics, alpha, beta, 2^beta and |x|^alpha * 2^beta
# are fp64 ops; float_quantize quantises the fp32 rounding of Y (qtorch's quantiser works on fp32
# words: the precision-16 branch's Y.float(); at precision 32 the dtype-generic extension, see
# include/smq.h SMQ_DTYPE_F64). Precision 32: the inverse in fp64. Precision 16: float_quantize
# returns half and the inverse runs in half as torch does — the 0-dim fp64 reciprocal of 2^beta
# enters the product as its fp32 value, the exponent 1/alpha is cast to half — times the fp64 signs.
# Powers and logarithms are the C library's (math.pow / math.log2, element by element: numpy's
# vectorised fp64 pow differs from libm in ~4 % of elements); the device's may differ by an ulp.
F64 = np.float64
_pow = np.frompyfunc(lambda a, b: _libm_pow(a, b), 2, 1)
_log2 = np.frompyfunc(lambda a: _libm_log2(a), 1, 1)


def _libm_pow(a, b):
    import math

    try:
        return math.pow(a, b)
    except (OverflowError, ValueError):
        return float(np.power(F64(a), F64(b)))


def _libm_log2(a):
    import math

    if a == 0.0 or a != a or a == float("inf"):
        return float(np.log2(F64(a))) if a != 0.0 else float("-inf")
    return math.log2(a)


def stats_f64(x):
    a = np.abs(np.asarray(x, dtype=F64))
    with np.errstate(all="ignore"):
        lg = np.where(a == F64(0), a, _log2(a).astype(F64))
    return derive_f64(float(np.mean(lg)), float(np.max(lg)))


def derive_f64(mu, m):
    mu, m = F64(mu), F64(m)
    with np.errstate(all="ignore"):
        alpha = (F64(1) / (m - mu)) * F64(15.0)
        beta = (-alpha) * mu
        bp2 = F64(_libm_pow(2.0, float(beta)))
        return dict(mu=mu, m=m, alpha=alpha, beta=beta, beta_pow2=bp2,
                    inv_beta_pow2=F64(1) / bp2, inv_alpha=F64(1) / alpha)


def transform_f64(x, st):
    a = np.abs(np.asarray(x, dtype=F64))
    with np.errstate(all="ignore"):
        return _pow(a, float(st["alpha"])).astype(F64) * st["beta_pow2"]


def roundtrip_f64(x, rand_bits, check_inf_flag=True, precision=32, st=None):
    """-> (y float64, st, Y float64, T float32 quantised codes' values)."""
    x = np.asarray(x, dtype=F64)
    st = stats_f64(x) if st is None else st
    Y = transform_f64(x, st)
    with np.errstate(all="ignore"):
        T = qf.float_quantize(Y.astype(F32), 5, 2, rand_bits, check_inf_flag)
        sgn = np.where(x > 0, F64(1), np.where(x < 0, F64(-1), F64(0)))
        if precision == 32:
            t2 = _pow(T.astype(F64) * st["inv_beta_pow2"], float(st["inv_alpha"])).astype(F64)
            return t2 * sgn, st, Y, T
        th = _r(T, "f16")
        t1 = _r(th * F32(st["inv_beta_pow2"]), "f16")
        ia = _r(F32(st["inv_alpha"]), "f16")
        t2 = _r(np.power(t1.astype(F64), F64(ia)).astype(F32), "f16")
        return t2.astype(F64) * sgn, st, Y, T
