"""Shared plumbing of the fixed-format float codecs (FP8 / FP16 / BF16 / FP32).

Reference: smart_compress/compress/{fp8,fp16,bf16,fp32}.py — each adds the float-quantise flags to
the base parser, logs a fixed bit-count ratio, and calls ``float_quantize(x, exp, man, hparams)``.
"""

from argparse import ArgumentParser

import torch

from ..util.pytorch import quantization as _q
from ..util.pytorch.quantization import add_float_quantize_args, float_quantize
from .base import CompressionAlgorithmBase


class FloatFormatCodec(CompressionAlgorithmBase):
    EXP_BITS: int = 0
    MAN_BITS: int = 0
    STORED_BITS: int = 32

    @staticmethod
    def add_argparse_args(parent_parser: ArgumentParser) -> ArgumentParser:
        return ArgumentParser(
            parents=[add_float_quantize_args(CompressionAlgorithmBase.add_argparse_args(parent_parser))],
            add_help=False,
        )

    def graph_safe(self, enable: bool = True, device=None):
        """hipGraph-capturable random stream (process-wide, see quantization.graph_safe)."""
        _q.graph_safe(enable, device)
        return self

    @torch.no_grad()
    def __call__(self, tensor: torch.Tensor, tag: str = None, **_):
        self.log_ratio(tag, tensor.numel(), 32, self.STORED_BITS)
        return float_quantize(tensor, exp=self.EXP_BITS, man=self.MAN_BITS, hparams=self.hparams)
