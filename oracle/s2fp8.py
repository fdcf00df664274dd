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
