"""FP32 (identity) codec: drop-in for smart_compress/compress/fp32.py:11-23."""

from argparse import ArgumentParser

import torch

from .base import CompressionAlgorithmBase


class FP32(CompressionAlgorithmBase):
    @staticmethod
    def add_argparse_args(parent_parser: ArgumentParser) -> ArgumentParser:
        return ArgumentParser(
            parents=[CompressionAlgorithmBase.add_argparse_args(parent_parser)], add_help=False
        )

    @torch.no_grad()
    def __call__(self, tensor: torch.Tensor, tag: str = None, **_):
        self.log_ratio(tag, tensor.numel(), 32, 32)
        return tensor
