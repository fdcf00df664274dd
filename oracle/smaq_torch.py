"""SmaQ round trip restated as the reference's own torch-CPU op sequence (test infrastructure).

TEST / BASELINE INFRASTRUCTURE ONLY: imported by tests/ and by bench.py's ``cpu_baseline`` leg (the
multi-threaded CPU time of the reference's algorithm on the GPU box's host cores, where the
reference itself is not present). Never part of the product path.

Follows smart_compress/compress/smart.py op for op with the default flags (full statistics,
unbiased std, stochastic rounding, fp32): statistics smart.py:100-108 / 130-134, the ``std == 0``
rule 151-152 (a host sync there too), z-score 154, outlier masks 155-157, scalars 159-161, ranges
162, scaling 164, ``_round_stochastic`` 93-98 with ``torch.rand_like``, de-quantisation 171-172,
de-normalisation 181-182, ``all_positive`` clamp (optimizer.py:58 callers). ``uniforms`` / ``stats``
inject the reference's recorded draws and statistics for bit-exact checks against tests/golden.
"""

from typing import Optional, Tuple

import torch


def roundtrip(x: torch.Tensor, num_bits_main: int = 6, num_bits_outlier: int = 8,
              thr: float = 1.0, thr_outlier: float = 2.5, all_positive: bool = False,
              uniforms: Optional[torch.Tensor] = None,
              stats: Optional[Tuple[float, float]] = None, num_samples: int = 0) -> torch.Tensor:
    """num_samples > 0: --use_sample_stats (smart.py:86-91: randperm(n)[:k], mean, biased std)."""
    r_out = ((2 ** (num_bits_outlier - 2)) - 1) / (thr_outlier - thr)  # Python doubles
    r_main = ((2 ** (num_bits_main - 2)) - 1) / thr
    if stats is None and num_samples > 0:
        k = min(x.numel(), num_samples)
        sample = x.view(-1)[torch.randperm(x.numel())[:k]]
        m, s = sample.mean(), sample.std(unbiased=False)
    elif stats is None:
        m, s = x.mean(), x.std()  # unbiased
    else:
        m, s = (torch.tensor(v, dtype=torch.float32) for v in stats)
    if s == 0:
        s = torch.ones_like(s)
    z = (x - m) / s.clamp(1e-38, 1e38)
    hi, lo = z > thr, z < -thr
    side = (hi * -thr) + (lo * thr)  # bool * Python float -> fp32, +-0 for mains
    r = torch.where(hi | lo, r_out, r_main)
    d = (z + side) * r
    u = torch.rand_like(d) if uniforms is None else uniforms
    f = d.floor()
    q = f + torch.relu(((d - f) - u) + 0.5).round()
    y = ((q / r) - side) * s + m
    return y.clamp_min(0.0) if all_positive else y
