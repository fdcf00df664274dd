"""qtorch 0.2.0 float quantisation restated in numpy uint32 arithmetic, plus the reference wrapper.

Third-party dependency absent from /root/reference (poetry.lock:773-781 pins qtorch 0.2.0; the
reference imports it at smart_compress/util/pytorch/quantization.py:3). Restated algorithm
(quant_cuda float_kernel_{stochastic,nearest}, bit_helper round_bitwise_*, clip_exponent):

  target = bits(x); e = ((target << 1) >> 24) - 127; min_exp = -(2^(E-1) - 2)
  if e < min_exp:   shift = sign(x) * 2^min_exp;  v = x + shift (fp32)
                    y = float(round(bits(v))) - shift
  else:             y = float(clip(round(target)))
  round(t) = (t + (r & M)) & ~M (stochastic)  |  (t + 2^(22-m)) & ~M (nearest),  M = 2^(23-m) - 1
  clip: biased exponent > 127 + 2^(E-1) - 1  ->  sign | max finite (saturation)

The random word r is qtorch's randint_like(x, INT_MAX) draw (CUDA) — only its low 23-m bits
matter. PARITY UNPINNED for this function: no reference test or fixture covers qtorch.
"""

import numpy as np

F32 = np.float32
U32 = np.uint32
FLT_MAX = np.finfo(np.float32).max
FLT_EPS = np.finfo(np.float32).eps


def _clip_exponent(exp_bits, man_bits, old, q):
    qexp = ((q << U32(1)) >> U32(24)).astype(np.int64)
    min_store = -((1 << (exp_bits - 1)) - 2) - 1 + 127
    max_store = ((1 << (exp_bits - 1)) - 1) + 127
    max_man = ((0xFFFFFFFF << 9) & 0xFFFFFFFF) >> 9 >> (23 - man_bits) << (23 - man_bits)
    max_num = U32((max_store << 23) | max_man)
    sign = old & U32(0x80000000)
    out = np.where(qexp > max_store, sign | max_num, q)
    min_num = U32((min_store << 23) & 0xFFFFFFFF)
    middle = U32(((min_store - 1) << 23) & 0xFFFFFFFF)
    under = qexp < min_store
    under_val = np.where((q & U32(0x7FFFFFFF)) > middle, sign | min_num, U32(0))
    return np.where(under & ~(qexp > max_store), under_val, out).astype(U32)


def quantize(x, exp_bits: int, man_bits: int, rand_bits=None, stochastic=True) -> np.ndarray:
    """qtorch float_quantize(x, exp, man, rounding) on float32 input (any shape)."""
    x = np.ascontiguousarray(x, dtype=F32)
    t = x.view(U32)
    mask = U32((1 << (23 - man_bits)) - 1)
    if stochastic:
        add = np.asarray(rand_bits, dtype=U32).reshape(x.shape) & mask
    else:
        add = U32(1 << (23 - man_bits - 1))
    texp = ((t << U32(1)) >> U32(24)).astype(np.int64) - 127
    min_exp = -((1 << (exp_bits - 1)) - 2)
    sub = texp < min_exp
    with np.errstate(all="ignore"):
        qn = ((t + add) & ~mask).astype(U32)
        qn = _clip_exponent(exp_bits, man_bits, t, qn)
        shift_bits = (U32(((127 + min_exp) << 23) & 0xFFFFFFFF) | (t & U32(0x80000000))).astype(U32)
        shift = shift_bits.view(F32)
        val = (x + shift).astype(F32)
        qs = ((val.view(U32) + add) & ~mask).astype(U32)
        ys = (qs.view(F32) - shift).astype(F32)
    return np.where(sub, ys, qn.view(F32)).astype(F32)


def max_value(exp_bits: int, man_bits: int) -> np.float32:
    """_get_max_value (quantization.py:138-150): nearest-quantised FLT_MAX."""
    return F32(quantize(np.array([FLT_MAX], dtype=F32), exp_bits, man_bits, stochastic=False)[0])


def check_inf(y: np.ndarray, exp_bits: int, man_bits: int) -> np.ndarray:
    """quantization.py:195-199: |y - max| <= FLT_EPS -> +inf."""
    mv = max_value(exp_bits, man_bits)
    with np.errstate(all="ignore"):
        hit = np.abs(y - mv) <= F32(FLT_EPS)
    out = y.copy()
    out[hit] = np.inf
    return out


def float_quantize(x, exp_bits, man_bits, rand_bits, check_inf_flag=True):
    """quantization.py:187-204 at precision 32 (stochastic)."""
    y = quantize(x, exp_bits, man_bits, rand_bits, stochastic=True)
    return check_inf(y, exp_bits, man_bits) if check_inf_flag else y
