"""SmaQ (smart_compress/compress/smart.py) restated op for op in numpy float32.

Every line is one IEEE-754 round-to-nearest float32 operation, in the reference's order; numpy does
not contract a*b+c into an FMA. Statistics are computed in float64 and rounded once to float32
(torch CPU's full-tensor mean/std agree with that to 0-1 ulp; tests pin the exact reference values).
"""

from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np

F32 = np.float32


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


def range_coef(n: int) -> np.float32:
    """1 / sqrt(2 * log(float32(n))) in float32 ops (smart.py:101-106)."""
    return F32(1) / np.sqrt(F32(2.0) * np.log(F32(n)))


def full_stats(x: np.ndarray, cfg: SmaqConfig) -> Tuple[np.float32, np.float32]:
    """(data.mean(), self._get_std(data)) — smart.py:131, 100-108 (unbiased std)."""
    x64 = x.astype(np.float64).ravel()
    mean = F32(np.mean(x64))
    if cfg.use_range_std_dev:
        rng = F32(x.max()) - F32(x.min())
        return mean, F32(rng * range_coef(x.size))
    d = x64 - np.mean(x64)
    var = float(np.dot(d, d)) / (x64.size - 1) if x64.size > 1 else float("nan")
    return mean, F32(np.sqrt(var))


def sampled_stats(x: np.ndarray, idx: np.ndarray, cfg: SmaqConfig):
    """smart.py:86-91: mean and biased std (or range-std) of x.view(-1)[idx]."""
    s = x.ravel()[np.asarray(idx, dtype=np.int64)]
    s64 = s.astype(np.float64)
    mean = F32(np.mean(s64))
    if cfg.use_range_std_dev:
        return mean, F32((F32(s.max()) - F32(s.min())) * range_coef(s.size))
    d = s64 - np.mean(s64)
    return mean, F32(np.sqrt(float(np.dot(d, d)) / s64.size))


def apply(x: np.ndarray, mean, std, cfg: SmaqConfig, uniforms: Optional[np.ndarray] = None,
          all_positive: bool = False, bn: Optional[Tuple[np.ndarray, np.ndarray]] = None):
    """smart.py:144-182 given (mean, std). Returns (y, is_outlier)."""
    x = np.asarray(x, dtype=F32)
    shape = x.shape
    mean, std = F32(mean), F32(std)
    thr = F32(cfg.main_std_dev_threshold)
    lo_c, hi_c = F32(cfg.clamped_range[0]), F32(cfg.clamped_range[1])
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
        z = (data - mean) / sc
        hi = z > thr
        lo = z < -thr
        o = hi | lo
        scal = np.where(hi, -thr, F32(0) * -thr) + np.where(lo, thr, F32(0) * thr)
        scal = scal.astype(F32)
        ranges = np.where(o, r_out, r_main).astype(F32)
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
        y = (q / ranges) - scal
        y = (y * std) + mean
        if bn is not None:  # smart.py:174-179
            y = (y * g) + b
        if all_positive:
            y = np.where(y < F32(0), F32(0), y)
    return y.astype(F32).reshape(shape), o.reshape(shape)


def roundtrip(x: np.ndarray, cfg: SmaqConfig, uniforms=None, sample_idx=None,
              all_positive=False, bn=None, stats=None):
    """Full smart.py:110-182. Returns (y, mean, std, n_outlier); n < min_size passes through."""
    if x.size < cfg.min_size:
        return x, None, None, 0
    if stats is not None:
        mean, std = stats
    elif cfg.use_sample_stats:
        mean, std = sampled_stats(x, sample_idx, cfg)
    else:
        mean, std = full_stats(x, cfg)
    y, o = apply(x, mean, std, cfg, uniforms, all_positive, bn)
    return y, mean, std, int(o.sum())
