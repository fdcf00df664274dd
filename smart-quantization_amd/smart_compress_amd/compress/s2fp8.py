"""S2FP8 codec: drop-in for smart_compress/compress/s2fp8.py:11-48.

Reference algorithm (per tensor): L = log2|x| with zeros as 0; mu = mean(L), m = max(L);
alpha = 15 / (m - mu), beta = -alpha * mu; Y = |x|^alpha * 2^beta; T = E5M2 stochastic
float_quantize(Y) (+ check_inf); y = (T * 2^-beta)^(1/alpha) * sign(x). Logged as 8 bits per element
plus 64 bits of per-tensor overhead (s2fp8.py:29).

On MI355X this is ``smq_s2fp8_roundtrip_f32``: a log2-domain statistics launch (last-arriving
workgroup finalises alpha, beta) and one fused transform/quantise/inverse launch.
"""

from argparse import ArgumentParser

import torch

from .. import _native as N
from ..util.pytorch.quantization import add_float_quantize_args, quant_rng
from .base import CompressionAlgorithmBase


class S2FP8(CompressionAlgorithmBase):
    @staticmethod
    def add_argparse_args(parent_parser: ArgumentParser) -> ArgumentParser:
        return ArgumentParser(
            parents=[add_float_quantize_args(CompressionAlgorithmBase.add_argparse_args(parent_parser))],
            add_help=False,
        )

    @torch.no_grad()
    def __call__(self, tensor: torch.Tensor, tag: str = None, **_):
        self.log_ratio(tag, tensor.numel(), 32, 8, overhead=64)
        if self.hparams.precision == 16:
            raise NotImplementedError("S2FP8 with precision=16 (half I/O) is not supported yet")
        N.require_device_f32(tensor, "S2FP8")
        x = tensor.contiguous()
        y = torch.empty_like(x)
        n = x.numel()
        if n == 0:
            return y
        ws = N.workspace("s2fp8", x.device, N.lib().smq_s2fp8_workspace_bytes(n))
        seed, offset = quant_rng().take(n)
        N.check(
            N.lib().smq_s2fp8_roundtrip_f32(
                x.data_ptr(), y.data_ptr(), n, 1 if self.hparams.float_quantize_check_inf else 0,
                None, seed, offset, None, ws.data_ptr(), ws.numel(), N.stream_ptr(x.device),
            ),
            "smq_s2fp8_roundtrip_f32",
        )
        return y
