"""SmaQ (smart_compress/compress/smart.py) restated op for op in numpy float32.

Every line is one IEEE-754 round-to-nearest float32 operation, in the reference's order; numpy does
not contract a*b+c into an FMA. Statistics are computed in float64 and rounded once to float32
(torch CPU's full-tensor mean/std agree with that to 0-1 ulp; tests pin the exact reference values).
"""

from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np

F32 = np.float32


def round_to(v, dtype: str = "f32"):
    """Round float32 value(s) to the input type and back (RN-even): 'f32' | 'f16' | 'bf16'.
    One input-type op = the float32 op + this rounding (exact: double rounding is innocuous when
    the wide format has >= 2p + 2 bits)."""
    a = np.asarray(v, dtype=F32)
    if dtype == "f16":
        with np.errstate(over="ignore"):
            return a.astype(np.float16).astype(F32)
    if dtype == "bf16":
        u = a.view(np.uint32).astype(np.uint64)
        r = ((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000).astype(np.uint32).view(F32)
        return np.where(np.isnan(a), a, r).astype(F32)
    return a


@dataclass
class SmaqConfig:
    """hparams of smart.py:11-70 and the constants of smart.py:72-84 (Python doubles)."""

    num_bits_main: int = 6
    num_bits_outlier: int = 8
    main_std_dev_threshold: float = 1.0
    outlier_std_dev_threshold: float = 2.5
    stochastic_rounding: bool = True
    use_sample_stats: bool = False
    num_samples: int = 16
    use_range_std_dev: bool = False
    min_size: int = 8
    precision: int = 32

    @property
    def range_outlier(self) -> float:  # smart.py:72-75
        return ((2 ** (self.num_bits_outlier - 2)) - 1) / (
            self.outlier_std_dev_threshold - self.main_std_dev_threshold)

    @property
    def range_normal(self) -> float:  # smart.py:76-78
        return ((2 ** (self.num_bits_main - 2)) - 1) / self.main_std_dev_threshold

    @property
    def clamped_range(self) -> Tuple[float, float]:  # smart.py:80-84
        return (1e-4, 1e4) if self.precision == 16 else (1e-38, 1e38)


def range_coef(n: int, dtype: str = "f32") -> np.float32:
    """1 / sqrt(2 * log(T(n))) with every op in the data's type T (smart.py:101-106)."""
    with np.errstate(all="ignore"):
        t = round_to(F32(n), dtype)
        t = round_to(np.log(t), dtype)
        t = round_to(F32(2.0) * t, dtype)
        t = round_to(np.sqrt(t), dtype)
        return F32(round_to(F32(1) / t, dtype))


def full_stats(x: np.ndarray, cfg: SmaqConfig, dtype: str = "f32") -> Tuple[np.float32, np.float32]:
    """(data.mean(), self._get_std(data)) — smart.py:131, 100-108 (unbiased std); for half data
    the 0-dim results are rounded to the data's type (through float32, as torch does)."""
    x64 = x.astype(np.float64).ravel()
    mean = F32(round_to(F32(np.mean(x64)), dtype))
    if cfg.use_range_std_dev:
        rng = round_to(F32(x.max()) - F32(x.min()), dtype)
        return mean, F32(round_to(rng * range_coef(x.size, dtype), dtype))
    d = x64 - np.mean(x64)
    var = float(np.dot(d, d)) / (x64.size - 1) if x64.size > 1 else float("nan")
    return mean, F32(round_to(F32(np.sqrt(var)), dtype))


def sampled_stats(x: np.ndarray, idx: np.ndarray, cfg: SmaqConfig, dtype: str = "f32"):
    """smart.py:86-91: mean and biased std (or range-std) of x.view(-1)[idx]."""
    s = x.ravel()[np.asarray(idx, dtype=np.int64)]
    s64 = s.astype(np.float64)
    mean = F32(round_to(F32(np.mean(s64)), dtype))
    if cfg.use_range_std_dev:
        rng = round_to(F32(s.max()) - F32(s.min()), dtype)
        return mean, F32(round_to(rng * range_coef(s.size, dtype), dtype))
    d = s64 - np.mean(s64)
    return mean, F32(round_to(F32(np.sqrt(float(np.dot(d, d)) / s64.size)), dtype))


def codes(x: np.ndarray, mean, std, cfg: SmaqConfig, uniforms: Optional[np.ndarray] = None,
          bn: Optional[Tuple[np.ndarray, np.ndarray]] = None, dtype: str = "f32"):
    """smart.py:144-169 given (mean, std): the integer-valued codes q and the outlier sides.
    Returns (q, hi, lo, std) with std after the ==0 rule (smart.py:151-152)."""
    x = np.asarray(x, dtype=F32)
    shape = x.shape
    mean, std = F32(mean), F32(std)
    thr = F32(cfg.main_std_dev_threshold)
    zt = "f32" if bn is not None else dtype  # fp32 BN parameters promote the data to fp32
    cthr = F32(round_to(thr, zt))
    lo_c = F32(round_to(F32(cfg.clamped_range[0]), dtype))
    hi_c = F32(round_to(F32(cfg.clamped_range[1]), dtype))
    r_out, r_main = F32(cfg.range_outlier), F32(cfg.range_normal)
    data = x
    if bn is not None:  # smart.py:144-149, per channel of dim 1
        g, b = [np.asarray(t, dtype=F32).reshape((1, -1, 1, 1)) for t in bn]
        data = (data - b) / g
    if std == F32(0):  # smart.py:151-152
        std = F32(1)
    sc = std
    if sc < lo_c:
        sc = lo_c
    if sc > hi_c:
        sc = hi_c
    with np.errstate(all="ignore"):
        z = round_to(round_to(data - mean, zt) / sc, zt)
        hi = z > cthr
        lo = z < -cthr
        scal, ranges = _scalars_ranges(hi, lo, thr, r_main, r_out)
        d = (z + scal) * ranges
        if cfg.stochastic_rounding:  # smart.py:93-98
            u = np.asarray(uniforms, dtype=F32).reshape(shape)
            f = np.floor(d)
            t = (d - f) - u
            t = t + F32(0.5)
            t = np.where(t < F32(0), F32(0), t).astype(F32)
            q = f + np.rint(t)
        else:
            q = np.trunc(d)
    return q.astype(F32), hi, lo, std


def _scalars_ranges(hi, lo, thr, r_main, r_out):
    """smart.py:159-162: scalars = hi * -T + lo * T (bool * float: +-0 zero terms), ranges."""
    scal = np.where(hi, -thr, F32(0) * -thr) + np.where(lo, thr, F32(0) * thr)
    ranges = np.where(hi | lo, r_out, r_main)
    return scal.astype(F32), ranges.astype(F32)


def dequant(q, hi, lo, mean, std, cfg: SmaqConfig, all_positive: bool = False,
            bn: Optional[Tuple[np.ndarray, np.ndarray]] = None):
    """smart.py:171-182: (q / ranges - scalars) * std + mean (std after the ==0 rule)."""
    thr = F32(cfg.main_std_dev_threshold)
    scal, ranges = _scalars_ranges(hi, lo, thr, F32(cfg.range_normal), F32(cfg.range_outlier))
    mean, std = F32(mean), F32(std)
    with np.errstate(all="ignore"):
        y = (np.asarray(q, dtype=F32) / ranges) - scal
        y = (y * std) + mean
        if bn is not None:  # smart.py:174-179
            g, b = [np.asarray(t, dtype=F32).reshape((1, -1, 1, 1)) for t in bn]
            y = (y * g) + b
        if all_positive:
            y = np.where(y < F32(0), F32(0), y)
    return y.astype(F32)


def apply(x: np.ndarray, mean, std, cfg: SmaqConfig, uniforms: Optional[np.ndarray] = None,
          all_positive: bool = False, bn: Optional[Tuple[np.ndarray, np.ndarray]] = None,
          dtype: str = "f32"):
    """smart.py:144-182 given (mean, std). Returns (y, is_outlier). For dtype 'f16' / 'bf16' the
    z-score is computed in that type (x, mean, std hold values of it) and the rest in float32 —
    the reference's torch type promotion; the output is float32."""
    shape = np.shape(x)
    q, hi, lo, std1 = codes(x, mean, std, cfg, uniforms, bn, dtype)
    y = dequant(q, hi, lo, mean, std1, cfg, all_positive, bn)
    return y.reshape(shape), (hi | lo).reshape(shape)


def roundtrip(x: np.ndarray, cfg: SmaqConfig, uniforms=None, sample_idx=None,
              all_positive=False, bn=None, stats=None, dtype: str = "f32"):
    """Full smart.py:110-182. Returns (y, mean, std, n_outlier); n < min_size passes through."""
    if x.size < cfg.min_size:
        return x, None, None, 0
    if stats is not None:
        mean, std = stats
    elif cfg.use_sample_stats:
        mean, std = sampled_stats(x, sample_idx, cfg, dtype)
    else:
        mean, std = full_stats(x, cfg, dtype)
    y, o = apply(x, mean, std, cfg, uniforms, all_positive, bn, dtype)
    return y, mean, std, int(o.sum())


# ---- float64 data (smart.py:130-182 under torch's type flow for a float64 tensor) -------------------
# Statistics, z-score, rounding and de-quantisation are fp64 ops; the clamp bounds and the
# threshold the z-score is compared with are the Python doubles; the scalars (bool * float) and
# ranges (torch.where of two Python floats) are float32 tensors, so their fp32 values enter the
# fp64 chain. Each line is one IEEE fp64 op in the reference's order (numpy does not contract).
F64 = np.float64


def range_coef_f64(n: int) -> float:
    """1 / sqrt(2 * log(double(n))) (smart.py:103-105 with type_as(range_) = float64)."""
    return float(F64(1.0) / np.sqrt(F64(2.0) * np.log(F64(n))))


def full_stats_f64(x: np.ndarray, cfg: SmaqConfig) -> Tuple[float, float]:
    """(data.mean(), std) of float64 data: mean, unbiased std (or range-std), in fp64."""
    x = np.asarray(x, dtype=F64).ravel()
    mean = float(np.mean(x))
    if cfg.use_range_std_dev:
        return mean, float((F64(x.max()) - F64(x.min())) * F64(range_coef_f64(x.size)))
    d = x - np.mean(x)
    var = float(np.dot(d, d)) / (x.size - 1) if x.size > 1 else float("nan")
    return mean, float(np.sqrt(var))


def sampled_stats_f64(x: np.ndarray, idx: np.ndarray, cfg: SmaqConfig) -> Tuple[float, float]:
    """smart.py:86-91 on float64 data: mean and biased std (or range-std) of the samples."""
    s = np.asarray(x, dtype=F64).ravel()[np.asarray(idx, dtype=np.int64)]
    mean = float(np.mean(s))
    if cfg.use_range_std_dev:
        return mean, float((F64(s.max()) - F64(s.min())) * F64(range_coef_f64(s.size)))
    d = s - np.mean(s)
    return mean, float(np.sqrt(float(np.dot(d, d)) / s.size))


def codes_f64(x: np.ndarray, mean: float, std: float, cfg: SmaqConfig,
              uniforms: Optional[np.ndarray] = None,
              bn: Optional[Tuple[np.ndarray, np.ndarray]] = None):
    """smart.py:144-169 on float64 data: (q float64, hi, lo) — apply_f64's codes (the packed
    container's input)."""
    x = np.asarray(x, dtype=F64)
    shape = x.shape
    mean, std = F64(mean), F64(std)
    thr = F64(cfg.main_std_dev_threshold)
    sthr = F64(F32(cfg.main_std_dev_threshold))
    r_out, r_main = F64(F32(cfg.range_outlier)), F64(F32(cfg.range_normal))
    lo_c, hi_c = (F64(v) for v in cfg.clamped_range)
    data = x
    if bn is not None:
        g, b = [np.asarray(t, dtype=F64).reshape((1, -1, 1, 1)) for t in bn]
        data = (data - b) / g
    if std == F64(0):
        std = F64(1)
    sc = std
    if sc < lo_c:
        sc = lo_c
    if sc > hi_c:
        sc = hi_c
    with np.errstate(all="ignore"):
        z = (data - mean) / sc
        hi = z > thr
        lo = z < -thr
        scal = (np.where(hi, -sthr, F64(F32(0) * -F32(cfg.main_std_dev_threshold)))
                + np.where(lo, sthr, F64(F32(0) * F32(cfg.main_std_dev_threshold))))
        ranges = np.where(hi | lo, r_out, r_main)
        d = (z + scal) * ranges
        if cfg.stochastic_rounding:
            u = np.asarray(uniforms, dtype=F64).reshape(shape)
            f = np.floor(d)
            t = (d - f) - u
            t = t + F64(0.5)
            t = np.where(t < F64(0), F64(0), t)
            q = f + np.rint(t)
        else:
            q = np.trunc(d)
    return q.reshape(shape), hi.reshape(shape), lo.reshape(shape)


def dequant_f64(q, hi, lo, mean: float, std_dev: float, thr32: float, r_main32: float,
                r_out32: float, all_positive: bool = False, bn=None, channel=None):
    """smart.py:171-182 on float64 codes: (q / ranges) - scalars, * std + mean (std after the ==0
    rule), then * gamma + beta per channel, clamp_min(0)."""
    sthr = F64(F32(thr32))
    ranges = np.where(hi | lo, F64(F32(r_out32)), F64(F32(r_main32)))
    scal = (np.where(hi, -sthr, F64(F32(0) * -F32(thr32)))
            + np.where(lo, sthr, F64(F32(0) * F32(thr32))))
    with np.errstate(all="ignore"):
        y = (np.asarray(q, F64) / ranges) - scal
        y = (y * F64(std_dev)) + F64(mean)
        if bn is not None:
            y = (y * bn[0][channel]) + bn[1][channel]
        if all_positive:
            y = np.where(y < F64(0), F64(0), y)
    return y


def apply_f64(x: np.ndarray, mean: float, std: float, cfg: SmaqConfig,
              uniforms: Optional[np.ndarray] = None, all_positive: bool = False,
              bn: Optional[Tuple[np.ndarray, np.ndarray]] = None):
    """smart.py:144-182 on float64 data given (mean, std); returns (y float64, is_outlier)."""
    x = np.asarray(x, dtype=F64)
    shape = x.shape
    mean, std = F64(mean), F64(std)
    thr = F64(cfg.main_std_dev_threshold)             # compared in fp64 (a Python double)
    sthr = F64(F32(cfg.main_std_dev_threshold))       # the fp32 scalars tensor's value
    r_out, r_main = F64(F32(cfg.range_outlier)), F64(F32(cfg.range_normal))
    lo_c, hi_c = (F64(v) for v in cfg.clamped_range)
    data = x
    if bn is not None:
        g, b = [np.asarray(t, dtype=F64).reshape((1, -1, 1, 1)) for t in bn]
        data = (data - b) / g
    if std == F64(0):
        std = F64(1)
    sc = std
    if sc < lo_c:
        sc = lo_c
    if sc > hi_c:
        sc = hi_c
    with np.errstate(all="ignore"):
        z = (data - mean) / sc
        hi = z > thr
        lo = z < -thr
        scal = (np.where(hi, -sthr, F64(F32(0) * -F32(cfg.main_std_dev_threshold)))
                + np.where(lo, sthr, F64(F32(0) * F32(cfg.main_std_dev_threshold))))
        ranges = np.where(hi | lo, r_out, r_main)
        d = (z + scal) * ranges
        if cfg.stochastic_rounding:
            u = np.asarray(uniforms, dtype=F64).reshape(shape)
            f = np.floor(d)
            t = (d - f) - u
            t = t + F64(0.5)
            t = np.where(t < F64(0), F64(0), t)
            q = f + np.rint(t)
        else:
            q = np.trunc(d)
        y = (q / ranges) - scal
        y = (y * std) + mean
        if bn is not None:
            y = (y * g) + b
        if all_positive:
            y = np.where(y < F64(0), F64(0), y)
    return y.astype(F64).reshape(shape), (hi | lo).reshape(shape)


def uniforms_f64(seed: int, offset: int, n: int, start: int = 0) -> np.ndarray:
    """The counter RNG's fp64 uniforms (the same 24-bit values as the fp32 path)."""
    from . import rng as _rng

    return _rng.smaq_u24(seed, offset, n, start).astype(F64) * F64(2.0**-24)
